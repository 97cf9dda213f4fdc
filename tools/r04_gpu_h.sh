#!/bin/bash
# GPU box: what-if parity (class path with decoded pods, every NPT) and the cfg5
# step at 1M nodes for pass-1 nodes-per-thread 2 and 4.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04h}
timeout -k 10 500 python -u -m pytest tests/test_whatif_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_whatif.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/${T}_whatif.log | tail -30; tail -3 gpurun_out/${T}_whatif.log; [ $rc -ne 0 ] && exit $rc
for npt in 2 4; do
  KSG_WC_NPT=$npt timeout -k 10 300 python bench_whatif.py --cpu-pods 0 > gpurun_out/${T}_cfg5_npt$npt.json 2> gpurun_out/${T}_cfg5_npt$npt.err || { tail -5 gpurun_out/${T}_cfg5_npt$npt.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/${T}_cfg5_npt$npt.json').read().splitlines()[-1]);print($npt, d['value'], d['ms_per_step'], json.dumps(d.get('roofline'))[:300])"
done
