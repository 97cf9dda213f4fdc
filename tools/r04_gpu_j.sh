#!/bin/bash
# GPU box: preemption parity (staged node-grouped toggles) + latency at 50k nodes,
# window-variant parity at cfg2 width, the cfg2 line, then the cfg5 PMC passes.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04j}
timeout -k 10 500 python -u -m pytest tests/test_preempt_gpu.py tests/test_parity_gpu.py tests/test_cycle_gpu.py tests/test_plugin_api_gpu.py tests/test_events_gpu.py tests/test_edge_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/${T}_tests.log | tail -20; tail -2 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/bench_preempt.py --nodes 50000 --pods 8 > gpurun_out/${T}_preempt_bench.json 2> gpurun_out/${T}_preempt_bench.err || { tail -5 gpurun_out/${T}_preempt_bench.err; exit 1; }
cat gpurun_out/${T}_preempt_bench.json
for pf in 0 1 0 1; do
  KSG_WIN_PFIX=$pf timeout -k 10 200 python bench.py --extra "" --cpu-baseline 0 --steps 10 --warmup 2 > gpurun_out/${T}_cfg2_pf$pf.json 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/${T}_cfg2_pf$pf.json').read().splitlines()[-1]);print('cfg2 pfix $pf',d['value'],d['ms_per_step'],d['roofline']['kernel_avg_us'])"
done
KSG_WIN_PFIX=1 timeout -k 10 200 python tools/probe_fixup.py 5000 2048 > gpurun_out/${T}_probe_pf1.txt 2>&1 || exit 1
sed -n 7,17p gpurun_out/${T}_probe_pf1.txt; tail -3 gpurun_out/${T}_probe_pf1.txt
timeout -k 10 300 python tools/dropin_probe.py > gpurun_out/${T}_dropin.json 2> gpurun_out/${T}_dropin.err || { tail -5 gpurun_out/${T}_dropin.err; exit 1; }
cat gpurun_out/${T}_dropin.json
bash tools/pmc_whatif.sh r04 > gpurun_out/${T}_pmc_whatif.log 2>&1 || { tail -20 gpurun_out/${T}_pmc_whatif.log; exit 1; }
tail -20 gpurun_out/${T}_pmc_whatif.log
