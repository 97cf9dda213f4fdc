#!/bin/bash
# GPU box: split hand-over on by default — window-variant parity, then merge blocks
# off/on under it (cfg2 bench, alternating).
set -o pipefail
mkdir -p gpurun_out
T=r04t
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k "cfg2_large or persistent" > gpurun_out/${T}_parity.log 2>&1 || { tail -20 gpurun_out/${T}_parity.log; exit 1; }
tail -2 gpurun_out/${T}_parity.log
for rep in 1 2; do
  for mb in 0 1; do
    KSG_WIN_MB=$mb timeout -k 10 200 python bench.py --extra "" --cpu-baseline 0 --steps 10 --warmup 2 > gpurun_out/${T}_cfg2_mb${mb}_$rep.json 2>&1 || { tail -5 gpurun_out/${T}_cfg2_mb${mb}_$rep.json; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/${T}_cfg2_mb${mb}_$rep.json').read().splitlines()[-1]);print('mb',$mb,'rep',$rep,d['value'],d['roofline']['kernel_avg_us'])"
  done
done
