#!/bin/bash
# Round 5, first box: the whole -m gpu suite, the cfg4 persistent-chain stamps
# (fine slots), then the default bench line.  Each step under its own limit.
set -o pipefail
export TAG=${TAG:-r05a}
mkdir -p gpurun_out
export KSG_PROGRESS=gpurun_out/progress.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/${TAG:-r05a}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG:-r05a}_gputest.log; exit 1; }
tail -2 gpurun_out/${TAG:-r05a}_gputest.log
timeout -k 10 300 python tools/chain_stamps.py --pods 1200 > gpurun_out/${TAG:-r05a}_stamps.json 2> gpurun_out/${TAG:-r05a}_stamps.err || { tail -20 gpurun_out/${TAG:-r05a}_stamps.err; exit 1; }
cat gpurun_out/${TAG:-r05a}_stamps.json
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG:-r05a}_bench.json 2> gpurun_out/${TAG:-r05a}_bench.err || { tail -20 gpurun_out/${TAG:-r05a}_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/'+__import__('os').environ.get('TAG','r05a')+'_bench.json').read().splitlines()[-1])
print('cfg2', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])
print('dropin', d.get('dropin'))
for c in ('cfg3', 'cfg4', 'cfg5'):
    x = d.get(c, {})
    print(c, x.get('value'), x.get('ms_per_step'), x.get('us_per_pod'), (x.get('roofline') or {}).get('frac'), x.get('dropin'))
PY
