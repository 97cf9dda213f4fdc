#!/bin/bash
# Round 5: cycle / plugin-API / preemption / table-chain / static-window parity on
# the main build (static records beside the persistent loop, asynchronous class
# upload, setup fold, victim store), the C-ABI drop-in latency, then A/B benches: cfg2 + cfg3 for main,
# main with the records before the launch, and w512; cfg4 main.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r05k}
SKIP_TESTS=${SKIP_TESTS:-0}
M=kube-scheduler-simulator-p9_amd/libksg.so
[ "$SKIP_TESTS" = 1 ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_static_window_gpu.py tests/test_cycle_gpu.py tests/test_plugin_api_gpu.py tests/test_preempt_gpu.py tests/test_parity_gpu.py tests/test_edge_gpu.py -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
for c in 2 4; do
  timeout -k 10 300 python tools/dropin_c.py --cfg $c --out gpurun_out/${TAG}_dropin.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin_$c.err || { tail -20 gpurun_out/${TAG}_dropin_$c.err; exit 1; }
done
cat gpurun_out/${TAG}_dropin.jsonl
TAG=${TAG}_ab ARMS="main:KSG_LIB=$M before:KSG_LIB=$M,KSG_STATIC_OVERLAP=0" BENCH="python bench.py --extra 3 --cpu-baseline 0 --steps 10 --warmup 2" FIELDS="d['value'], d['roofline']['kernel_avg_us'], d['cfg3']['value'], d['cfg3']['roofline']['kernel_avg_us']" REPS=2 bash tools/gpu_ab.sh || exit 1
TAG=${TAG}_c4 ARMS="main:KSG_LIB=$M" BENCH="python bench.py --extra 4 --cpu-baseline 0 --steps 5 --warmup 1" FIELDS="d['cfg4']['us_per_pod']" REPS=2 bash tools/gpu_ab.sh
