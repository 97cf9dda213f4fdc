#!/bin/bash
# GPU box: window + view parity, the cfg2 window loop with the prefetched counters
# (prior step in the merges / in the replay), the drop-in latency with narrow view rows.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04l}
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_plugin_api_gpu.py tests/test_cycle_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
for pf in 0 1 0 1; do
  KSG_WIN_PFIX=$pf timeout -k 10 200 python bench.py --extra "" --cpu-baseline 0 --steps 10 --warmup 2 > gpurun_out/${T}_cfg2_pf$pf.json 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/${T}_cfg2_pf$pf.json').read().splitlines()[-1]);print('cfg2 pfix $pf',d['value'],d['ms_per_step'],d['roofline']['kernel_avg_us'],d['dropin'])"
done
for pf in 0 1; do
  KSG_WIN_PFIX=$pf timeout -k 10 200 python tools/probe_fixup.py 5000 2048 > gpurun_out/${T}_probe_pf$pf.txt 2>&1 || exit 1
  echo "== pfix $pf"; sed -n 14,17p gpurun_out/${T}_probe_pf$pf.txt
done
timeout -k 10 300 python tools/dropin_probe.py > gpurun_out/${T}_dropin.json 2> gpurun_out/${T}_dropin.err || { tail -5 gpurun_out/${T}_dropin.err; exit 1; }
cat gpurun_out/${T}_dropin.json
