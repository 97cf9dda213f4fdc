#!/bin/bash
# Round 5: preemption (victim store) + cycle-view (prefetched view) parity, the
# preemption latency bench, then the C-ABI drop-in latency for cfg2 and cfg4.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r05i}
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_preempt_gpu.py tests/test_cycle_gpu.py tests/test_plugin_api_gpu.py ${TESTS} -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
timeout -k 10 600 python tools/bench_preempt.py > gpurun_out/${TAG}_preempt.json 2> gpurun_out/${TAG}_preempt.err || { tail -20 gpurun_out/${TAG}_preempt.err; exit 1; }
cat gpurun_out/${TAG}_preempt.json
for c in 2 4; do
  timeout -k 10 300 python tools/dropin_c.py --cfg $c --out gpurun_out/${TAG}_dropin.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin_$c.err || { tail -20 gpurun_out/${TAG}_dropin_$c.err; exit 1; }
  KSG_VIEW_PREFETCH=0 timeout -k 10 300 python tools/dropin_c.py --cfg $c --out gpurun_out/${TAG}_dropin_noprefetch.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin_$c.err || { tail -20 gpurun_out/${TAG}_dropin_$c.err; exit 1; }
done
cat gpurun_out/${TAG}_dropin.jsonl gpurun_out/${TAG}_dropin_noprefetch.jsonl
