#!/bin/bash
# GPU box, a round's final build: the whole -m gpu suite, smoke(), the default
# bench line, then the C-ABI drop-in at cfg2 / cfg4 (tools/dropin_c.py).
#   TAG=r06_final bash tools/final_bench.sh
# Each step under its own time limit; the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-final}
if [ -z "$NO_TESTS" ]; then
  TAG=${TAG}_gputest LIMIT=${TEST_LIMIT:-900} bash tools/gpu_tests.sh || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
for c in ${DROPIN_CFGS-2 4}; do
  timeout -k 10 300 python tools/dropin_c.py --cfg $c --out gpurun_out/${TAG}_dropin.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin.err || { tail -20 gpurun_out/${TAG}_dropin.err; exit 1; }
done
[ -f gpurun_out/${TAG}_dropin.jsonl ] && cut -c1-240 gpurun_out/${TAG}_dropin.jsonl
python3 - <<PY
import json
d = json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1])
r = d['roofline']
print('cfg2', d['value'], d['ms_per_step'], r['kernel_avg_us'], r.get('traffic'), r['frac'])
print('dropin', d.get('dropin'))
for c in ('cfg3', 'cfg4', 'cfg5'):
    x = d.get(c) or {}
    print(c, x.get('value'), x.get('ms_per_step'), x.get('us_per_pod'), (x.get('roofline') or {}).get('kernel_avg_us'),
          (x.get('roofline') or {}).get('frac'))
PY
