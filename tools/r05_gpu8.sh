#!/bin/bash
# Round 5: class-table paths (fused upload, staged k_pc_build), zero-copy program
# placement, the cycle summary from the prefetched view and the packed lookup plan
# — parity of every table-chain / cycle path, the C-ABI drop-in latency and its
# kernel trace at cfg4, then a cfg4 A/B of the packed plan against libksg_base.so.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05o}
M=kube-scheduler-simulator-p9_amd/libksg.so
B=kube-scheduler-simulator-p9_amd/libksg_base.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_cycle_gpu.py tests/test_plugin_api_gpu.py tests/test_events_gpu.py tests/test_parity_gpu.py tests/test_edge_gpu.py tests/test_preempt_gpu.py tests/test_distributed.py tests/test_fullsize_gpu.py::test_cfg4_full_size_matches_oracle -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
for c in 2 4; do
  timeout -k 10 300 python tools/dropin_c.py --cfg $c --out gpurun_out/${TAG}_dropin.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin_$c.err || { tail -20 gpurun_out/${TAG}_dropin_$c.err; exit 1; }
done
cat gpurun_out/${TAG}_dropin.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_dropin_kt -o run -- python3 tools/dropin_c.py --cfg 4 --count 100 > gpurun_out/${TAG}_dropin_kt.log 2>&1 || { tail -20 gpurun_out/${TAG}_dropin_kt.log; exit 1; }
find gpurun_out/${TAG}_dropin_kt -name "*kernel_stats.csv" -exec head -12 {} \;
TAG=${TAG}_ab ARMS="packed:KSG_LIB=$M base:KSG_LIB=$B" BENCH="python bench.py --extra 4 --cpu-baseline 0 --steps 5 --warmup 1" FIELDS="d['cfg4']['us_per_pod'], d['cfg4']['roofline']['kernel_avg_us']" REPS=3 bash tools/gpu_ab.sh
