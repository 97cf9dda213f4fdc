#!/bin/bash
# GPU box: view parity (direct / copy) and the drop-in latency at cfg4 (both view paths).
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04m}
timeout -k 10 300 python -u -m pytest tests/test_plugin_api_gpu.py tests/test_cycle_gpu.py tests/test_edge_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
for cp in 0 1 0; do
  KSG_VIEW_COPY=$cp timeout -k 10 300 python tools/dropin_probe.py > gpurun_out/${T}_dropin_copy$cp.json 2> gpurun_out/${T}_dropin.err || { tail -5 gpurun_out/${T}_dropin.err; exit 1; }
  echo "copy=$cp $(cat gpurun_out/${T}_dropin_copy$cp.json)"
done
