#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04n}
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k "cfg2 or tight or selected" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/probe_fixup.py 5000 2048 > gpurun_out/${T}_probe.txt 2>&1 || exit 1
sed -n 1,2p gpurun_out/${T}_probe.txt; sed -n 14,17p gpurun_out/${T}_probe.txt
for i in 1 2; do
timeout -k 10 200 python bench.py --extra "" --cpu-baseline 0 --steps 10 --warmup 2 > gpurun_out/${T}_cfg2_$i.json 2>&1 || exit 1
python -c "import json;d=json.loads(open('gpurun_out/${T}_cfg2_$i.json').read().splitlines()[-1]);print('cfg2',d['value'],d['ms_per_step'],d['roofline']['kernel_avg_us'])"
done
