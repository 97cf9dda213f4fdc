#!/bin/bash
# GPU box: split hand-over of the window loop (KSG_WIN_SPLIT) — parity of every
# window variant at cfg2 width, then the cfg2 bench alternating off/on, then the probe.
set -o pipefail
mkdir -p gpurun_out
T=r04s
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k "cfg2_large" > gpurun_out/${T}_parity.log 2>&1 || { tail -20 gpurun_out/${T}_parity.log; exit 1; }
tail -2 gpurun_out/${T}_parity.log
for rep in 1 2; do
  for sp in 0 1; do
    KSG_WIN_SPLIT=$sp timeout -k 10 200 python bench.py --extra "" --cpu-baseline 0 --steps 10 --warmup 2 > gpurun_out/${T}_cfg2_sp${sp}_$rep.json 2>&1 || { tail -5 gpurun_out/${T}_cfg2_sp${sp}_$rep.json; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/${T}_cfg2_sp${sp}_$rep.json').read().splitlines()[-1]);print('split',$sp,'rep',$rep,d['value'],d['roofline']['kernel_avg_us'])"
  done
done
KSG_WIN_SPLIT=1 timeout -k 10 200 python tools/probe_fixup.py 5000 2048 > gpurun_out/${T}_probe_sp1.txt 2>&1 || exit 1
grep -h "period\|fixup duration\|W-1 end\|last merge" gpurun_out/${T}_probe_sp1.txt
