#!/bin/bash
# Round 5: k_view writes each message slot into the host block as it claims it
# (KSG_VIEW_SLOTS_DIRECT; no last-block copy of the table).  View / class-table
# parity, then the C-ABI drop-in latency at cfg4 per arm (three alternations),
# cfg2, kernel traces per arm, and the bench's cfg4 / cfg2 lines on this build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05u}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_plugin_api_gpu.py tests/test_cycle_gpu.py tests/test_parity_gpu.py -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
for r in 1 2 3; do
  for a in 1 0; do
    KSG_VIEW_SLOTS_DIRECT=$a timeout -k 10 300 python tools/dropin_c.py --cfg 4 --out gpurun_out/${TAG}_dropin_sd$a.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin.err || { tail -20 gpurun_out/${TAG}_dropin.err; exit 1; }
  done
done
for a in 1 0; do
  KSG_VIEW_SLOTS_DIRECT=$a timeout -k 10 300 python tools/dropin_c.py --cfg 2 --out gpurun_out/${TAG}_dropin_cfg2_sd$a.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin.err || { tail -20 gpurun_out/${TAG}_dropin.err; exit 1; }
done
for a in 1 0; do
  export KSG_VIEW_SLOTS_DIRECT=$a
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_sd$a -o run -- python3 tools/dropin_c.py --cfg 4 --count 100 > gpurun_out/${TAG}_kt_sd$a.log 2>&1 || { tail -20 gpurun_out/${TAG}_kt_sd$a.log; exit 1; }
done
unset KSG_VIEW_SLOTS_DIRECT
timeout -k 10 600 python bench.py --cpu-baseline 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
for a in 1 0; do echo "== sd$a"; cut -c1-120 gpurun_out/${TAG}_dropin_sd$a.jsonl; done
python3 -c "
import json;d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1])
print(d['value'], d.get('ms_per_step'), d.get('dropin'))
for c in ('cfg3','cfg4','cfg5'):
    x=d.get(c) or {}; print(c, x.get('value'), x.get('us_per_pod'), x.get('dropin'))"
