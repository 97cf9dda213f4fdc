#!/bin/bash
# GPU box: A/B of KSG_STAGE (candidate ranks staged in LDS): 4 (A, libksg.so) vs 2 or 8
# (B, libksg_b.so) under the split hand-over, cfg2 bench alternating, B's parity.
set -o pipefail
mkdir -p gpurun_out
T=r04v
for rep in 1 2; do
  for v in a b; do
    if [ $v = a ]; then L=kube-scheduler-simulator-p9_amd/libksg.so; else L=kube-scheduler-simulator-p9_amd/libksg_b.so; fi
    KSG_LIB=$L timeout -k 10 200 python bench.py --extra "" --cpu-baseline 0 --steps 10 --warmup 2 > gpurun_out/${T}_cfg2_${v}_$rep.json 2>&1 || { tail -5 gpurun_out/${T}_cfg2_${v}_$rep.json; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/${T}_cfg2_${v}_$rep.json').read().splitlines()[-1]);print('$v',$rep,d['value'],d['roofline']['kernel_avg_us'])"
  done
done
KSG_LIB=kube-scheduler-simulator-p9_amd/libksg_b.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k "cfg2_large" > gpurun_out/${T}_parity.log 2>&1; rc=$?
tail -2 gpurun_out/${T}_parity.log
exit $rc
