#!/bin/bash
# GPU box: cycle-view parity (direct / copy) and the drop-in latency at cfg4, then
# the cfg3 / cfg4 profiles.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04k}
timeout -k 10 300 python -u -m pytest tests/test_plugin_api_gpu.py tests/test_cycle_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
for cp in 0 1; do
  KSG_VIEW_COPY=$cp timeout -k 10 300 python tools/dropin_probe.py > gpurun_out/${T}_dropin_copy$cp.json 2> gpurun_out/${T}_dropin.err || { tail -5 gpurun_out/${T}_dropin.err; exit 1; }
  cat gpurun_out/${T}_dropin_copy$cp.json
done
bash tools/prof_config.sh 4 --nodes 50000 --existing 200000 --pods 1000 > gpurun_out/r04_cfg4_kernel_stats.csv || exit 1
bash tools/prof_config.sh 3 --nodes 15000 --pods 2000 > gpurun_out/r04_cfg3_kernel_stats.csv || exit 1
bash tools/pmc_config.sh 4 r04 --nodes 50000 --existing 200000 --pods 600 > /dev/null || exit 1
bash tools/pmc_config.sh 3 r04 --nodes 15000 --pods 2000 > /dev/null || exit 1
echo profiles done
