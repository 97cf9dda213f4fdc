#!/bin/bash
# GPU box (round 4, step a): parity of the persistent chain (parity slots, lag,
# fallback, abort), the persistent window loop and the device cycle view; then
# the cfg2 window period (persistent vs per-window launches, eval tile sizes) and
# the cfg4 line with drop-in latency.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_plugin_api_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1
rc=$?; tail -8 gpurun_out/r04a_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0; do
  export KSG_WIN_RUN=$v
  timeout -k 10 200 python bench.py --extra "" --cpu-baseline 0 --steps 10 --warmup 2 > gpurun_out/r04a_cfg2_run$v.json 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r04a_cfg2_run$v.json').read().splitlines()[-1]);print('winrun',$v,d['value'],d['ms_per_step'],d['roofline']['kernel_avg_us'],d['dropin'])"
done
unset KSG_WIN_RUN
for npt in 2 5; do
  export KSG_WIN_NPT=$npt
  timeout -k 10 200 python bench.py --extra "" --cpu-baseline 0 --steps 10 --warmup 2 > gpurun_out/r04a_cfg2_npt$npt.json 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r04a_cfg2_npt$npt.json').read().splitlines()[-1]);print('npt',$npt,d['value'],d['ms_per_step'],d['roofline']['kernel_avg_us'])"
done
unset KSG_WIN_NPT
timeout -k 10 300 python bench.py --extra 4 --cpu-baseline 0 --steps 3 > gpurun_out/r04a_bench4.json 2> gpurun_out/r04a_bench4.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/r04a_bench4.json').read().splitlines()[-1]);c=d['cfg4'];print('cfg4',c['us_per_pod'],c['dropin'])"
timeout -k 10 300 python tools/cfg4_ab.py --pods 2000 > gpurun_out/r04a_cfg4_ab.json 2> gpurun_out/r04a_cfg4_ab.err || exit 1
head -20 gpurun_out/r04a_cfg4_ab.json
