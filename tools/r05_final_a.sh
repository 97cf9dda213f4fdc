#!/bin/bash
# Round 5 final build, part A: the default bench line (cfg2 headline + cfg3/4/5 legs
# + CPU baselines + drop-in), then the headline's kernel trace and HBM-traffic PMC
# passes (tools/headline_profile.sh).  Results under gpurun_out/ (copy to profiles/).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05_final}
timeout -k 10 900 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python - <<PY
import json
d = json.loads(open('gpurun_out/${TAG}_bench.json').read().splitlines()[-1])
print('cfg2', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline'].get('traffic'), d['roofline']['frac'])
print('dropin', d.get('dropin'))
print('cpu', d['cpu_baseline']['value'])
for c in ('cfg3', 'cfg4', 'cfg5'):
    x = d.get(c) or {}
    print(c, x.get('value'), x.get('ms_per_step'), x.get('us_per_pod'), (x.get('roofline') or {}).get('kernel_avg_us'), (x.get('roofline') or {}).get('frac'))
PY
bash tools/headline_profile.sh r05 > gpurun_out/r05_headline.log 2>&1 || { tail -20 gpurun_out/r05_headline.log; exit 1; }
tail -3 gpurun_out/r05_headline.log
