#!/bin/bash
# Round 5: the owner's deferred node-level assume in k_chain_run — persistent-chain
# parity (every variant, incl. no-defer) and full-size cfg4, then a cfg4 A/B
# against libksg_base.so (the build before it) and block 0's stamps; the view
# kernel's LDS-staged 16-byte writes through the C-ABI drop-in latency.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05r}
M=kube-scheduler-simulator-p9_amd/libksg.so
B=kube-scheduler-simulator-p9_amd/libksg_base.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_parity_gpu.py tests/test_fullsize_gpu.py::test_cfg4_full_size_matches_oracle tests/test_cycle_gpu.py tests/test_plugin_api_gpu.py -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
TAG=${TAG}_ab ARMS="defer:KSG_LIB=$M base:KSG_LIB=$B" BENCH="python bench.py --extra 4 --cpu-baseline 0 --steps 5 --warmup 1" FIELDS="d['cfg4']['us_per_pod'], d['cfg4']['roofline']['kernel_avg_us']" REPS=3 bash tools/gpu_ab.sh || exit 1
timeout -k 10 300 python tools/chain_stamps.py --pods 1200 > gpurun_out/${TAG}_stamps.json 2> gpurun_out/${TAG}_stamps.err || { tail -20 gpurun_out/${TAG}_stamps.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_stamps.json'));print(json.dumps(d['k_chain_run_us_since_pod_start_block0']));print(d.get('k_chain_run_latest_block_partial_us'))"
for c in 2 4; do
  timeout -k 10 300 python tools/dropin_c.py --cfg $c --out gpurun_out/${TAG}_dropin.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin_$c.err || { tail -20 gpurun_out/${TAG}_dropin_$c.err; exit 1; }
done
cat gpurun_out/${TAG}_dropin.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_dropin_kt -o run -- python3 tools/dropin_c.py --cfg 4 --count 100 > gpurun_out/${TAG}_dropin_kt.log 2>&1 || { tail -20 gpurun_out/${TAG}_dropin_kt.log; exit 1; }
find gpurun_out/${TAG}_dropin_kt -name "*kernel_stats.csv" -exec head -6 {} \;
