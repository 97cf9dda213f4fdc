#!/bin/bash
# Round 5: fused class upload (k_upload) + wave-aggregated k_pc_build — parity of
# every class-table path (cycles, plugin API, events, tables, full-size cfg4),
# then the C-ABI drop-in latency and its kernel trace at cfg4.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05m}
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_cycle_gpu.py tests/test_plugin_api_gpu.py tests/test_events_gpu.py tests/test_parity_gpu.py tests/test_edge_gpu.py tests/test_preempt_gpu.py tests/test_fullsize_gpu.py::test_cfg4_full_size_matches_oracle -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
for c in 2 4; do
  timeout -k 10 300 python tools/dropin_c.py --cfg $c --out gpurun_out/${TAG}_dropin.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin_$c.err || { tail -20 gpurun_out/${TAG}_dropin_$c.err; exit 1; }
done
cat gpurun_out/${TAG}_dropin.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_dropin_kt -o run -- python3 tools/dropin_c.py --cfg 4 --count 100 > gpurun_out/${TAG}_dropin_kt.log 2>&1 || { tail -20 gpurun_out/${TAG}_dropin_kt.log; exit 1; }
find gpurun_out/${TAG}_dropin_kt -name "*kernel_stats.csv" -exec cat {} \;
