#!/bin/bash
# Round 5: vectorised program placement — cycle / plugin-API / event parity, then
# the C-ABI drop-in latency (two runs per config) and its kernel trace at cfg2 and cfg4.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05q}
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_cycle_gpu.py tests/test_plugin_api_gpu.py tests/test_events_gpu.py tests/test_preempt_gpu.py -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
for rep in 1 2; do
  for c in 2 4; do
    timeout -k 10 300 python tools/dropin_c.py --cfg $c --out gpurun_out/${TAG}_dropin.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin_$c.err || { tail -20 gpurun_out/${TAG}_dropin_$c.err; exit 1; }
  done
done
cat gpurun_out/${TAG}_dropin.jsonl
for c in 2 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_dropin_kt$c -o run -- python3 tools/dropin_c.py --cfg $c --count 100 > gpurun_out/${TAG}_dropin_kt$c.log 2>&1 || { tail -20 gpurun_out/${TAG}_dropin_kt$c.log; exit 1; }
  find gpurun_out/${TAG}_dropin_kt$c -name "*kernel_stats.csv" -exec head -8 {} \;
done
