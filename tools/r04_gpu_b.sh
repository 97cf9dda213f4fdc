#!/bin/bash
# GPU box: cfg2 window period — persistent window loop (with / without dedicated
# merge blocks) vs per-window launches — with the fixup / eval stamps
# (tools/probe_fixup.py); parity of the window tests first.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04b}
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_plugin_api_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
for v in "1 1" "1 0" "0 1"; do
  set -- $v
  export KSG_WIN_RUN=$1 KSG_WIN_MB=$2
  timeout -k 10 200 python bench.py --extra "" --cpu-baseline 0 --steps 10 --warmup 2 > gpurun_out/${T}_cfg2_run$1$2.json 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/${T}_cfg2_run$1$2.json').read().splitlines()[-1]);print('winrun',$1,'mb',$2,d['value'],d['ms_per_step'],d['roofline']['kernel_avg_us'],d['dropin']['view_us'])"
  timeout -k 10 200 python tools/probe_fixup.py 5000 2048 > gpurun_out/${T}_probe_run$1$2.txt 2>&1 || exit 1
done
head -22 gpurun_out/${T}_probe_run11.txt
