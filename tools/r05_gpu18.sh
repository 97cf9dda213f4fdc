#!/bin/bash
# Round 5: the drop-in cycle's classes registered and built before the pod's
# program is compiled (KSG_CLASSES_EARLY), and ROCTx ranges of the host phases
# (KSG_ROCTX=1, rocprofv3 --marker-trace).  Cycle / view parity with the early
# classes, the C-ABI drop-in A/B at cfg4 (three alternations), a marker + kernel
# trace of the drop-in run.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05v}
KSG_CLASSES_EARLY=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_plugin_api_gpu.py tests/test_cycle_gpu.py -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
for r in 1 2 3; do
  for a in 1 0; do
    KSG_CLASSES_EARLY=$a timeout -k 10 300 python tools/dropin_c.py --cfg 4 --out gpurun_out/${TAG}_dropin_ce$a.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin.err || { tail -20 gpurun_out/${TAG}_dropin.err; exit 1; }
  done
done
export KSG_ROCTX=1
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_markers -o run -- python3 tools/dropin_c.py --cfg 4 --count 100 > gpurun_out/${TAG}_markers.log 2>&1 || { tail -20 gpurun_out/${TAG}_markers.log; exit 1; }
unset KSG_ROCTX
for a in 1 0; do echo "== ce$a"; cut -c1-120 gpurun_out/${TAG}_dropin_ce$a.jsonl; done
find gpurun_out/${TAG}_markers -name "*.csv" | head
