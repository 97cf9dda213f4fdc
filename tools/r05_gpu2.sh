#!/bin/bash
# Round 5 iteration box: table-chain / static-record parity subset, cfg4 stamps,
# then the bench line with cfg3 + cfg4 (no CPU baselines).  Each step limited.
set -o pipefail
export TAG=${TAG:-r05c}
mkdir -p gpurun_out
export KSG_PROGRESS=gpurun_out/progress.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread ${TESTS:-tests/test_parity_gpu.py tests/test_static_window_gpu.py tests/test_edge_gpu.py tests/test_fullsize_gpu.py::test_cfg4_full_size_matches_oracle} -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -2 gpurun_out/${TAG}_gputest.log
timeout -k 10 300 python tools/chain_stamps.py --pods 1200 > gpurun_out/${TAG}_stamps.json 2> gpurun_out/${TAG}_stamps.err || { tail -20 gpurun_out/${TAG}_stamps.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_stamps.json'));print(json.dumps(d['us_avg_block0']));print(json.dumps({k:v for k,v in d.items() if k.startswith('k_chain') or k.startswith('k_eval')}))"
timeout -k 10 600 python -u bench.py --extra ${EXTRA:-3,4} --cpu-baseline 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python - <<'PY'
import json, os
d = json.loads(open('gpurun_out/%s_bench.json' % os.environ['TAG']).read().splitlines()[-1])
print('cfg2', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])
for c in ('cfg3', 'cfg4', 'cfg5'):
    x = d.get(c) or {}
    print(c, x.get('value'), x.get('ms_per_step'), x.get('us_per_pod'), (x.get('roofline') or {}).get('kernel_avg_us'),
          ((x.get('roofline') or {}).get('other_kernels') or {}).get('k_static', {}).get('total_ms'))
PY
