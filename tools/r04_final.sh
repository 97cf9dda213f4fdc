#!/bin/bash
# GPU box: the default bench line (cfg2 headline + cfg3/4/5 + CPU baselines) on the final build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r04_final_bench.json 2> gpurun_out/r04_final_bench.err || { tail -20 gpurun_out/r04_final_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r04_final_bench.json').read().splitlines()[-1])
print('cfg2', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline'].get('traffic'), d['roofline']['frac'])
print('dropin', d.get('dropin'))
print('cpu', d['cpu_baseline']['value'])
for c in ('cfg3', 'cfg4', 'cfg5'):
    x = d.get(c, {})
    print(c, x.get('value'), x.get('ms_per_step'), x.get('us_per_pod'), (x.get('roofline') or {}).get('frac'), (x.get('cpu_baseline') or {}).get('value'), x.get('dropin'))
PY
