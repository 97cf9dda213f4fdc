#!/bin/bash
# GPU box: cfg2 window period, persistent window loop vs per-window launches, with
# the fixup / eval stamps of both (tools/probe_fixup.py).
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04b}
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "cfg2 or tight or batch or golden or known" > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0; do
  export KSG_WIN_RUN=$v
  timeout -k 10 200 python bench.py --extra "" --cpu-baseline 0 --steps 10 --warmup 2 > gpurun_out/${T}_cfg2_run$v.json 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/${T}_cfg2_run$v.json').read().splitlines()[-1]);print('winrun',$v,d['value'],d['ms_per_step'],d['roofline']['kernel_avg_us'],d['dropin']['view_us'])"
  timeout -k 10 200 python tools/probe_fixup.py 5000 2048 > gpurun_out/${T}_probe_run$v.txt 2>&1 || exit 1
done
cat gpurun_out/${T}_probe_run1.txt
