#!/bin/bash
# Round 5, final build: the whole -m gpu suite, smoke(), the default bench line,
# and the C-ABI drop-in at cfg2 / cfg4.  The first failure ends it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r05_final_c LIMIT=900 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_final_c_smoke.log 2>&1 || { tail -20 gpurun_out/r05_final_c_smoke.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/r05_final_c_bench.json 2> gpurun_out/r05_final_c_bench.err || { tail -20 gpurun_out/r05_final_c_bench.err; exit 1; }
for c in 2 4; do
  timeout -k 10 300 python tools/dropin_c.py --cfg $c --out gpurun_out/r05_final_c_dropin.jsonl > /dev/null 2> gpurun_out/r05_final_c_dropin.err || { tail -20 gpurun_out/r05_final_c_dropin.err; exit 1; }
done
cut -c1-200 gpurun_out/r05_final_c_dropin.jsonl
python3 -c "
import json;d=json.loads(open('gpurun_out/r05_final_c_bench.json').read().strip().splitlines()[-1])
print(d['value'], d.get('ms_per_step'), d.get('dropin'))
for c in ('cfg3','cfg4','cfg5'):
    x=d.get(c) or {}; print(c, x.get('value'), x.get('us_per_pod'), x.get('ms_per_step'))"
