#!/bin/bash
# GPU box (round 4, step a): persistent-chain parity (parity slots, lag, fallback,
# abort), the device cycle view, the cfg4 line (drop-in latency), and the cfg2
# window period against eval tile sizes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py tests/test_plugin_api_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "persistent or view or extension" > gpurun_out/r04a_persist.log 2>&1
rc=$?; tail -8 gpurun_out/r04a_persist.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --extra 4 --cpu-baseline 0 --steps 5 > gpurun_out/r04a_bench4.json 2> gpurun_out/r04a_bench4.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/r04a_bench4.json').read().splitlines()[-1]);print('cfg2',d['value'],d['roofline']['kernel_avg_us'],d['dropin']);c=d['cfg4'];print('cfg4',c['us_per_pod'],c['dropin'])"
for npt in 2 3 5; do
  export KSG_WIN_NPT=$npt
  timeout -k 10 200 python bench.py --extra "" --cpu-baseline 0 --steps 10 --warmup 2 > gpurun_out/r04a_cfg2_npt$npt.json 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r04a_cfg2_npt$npt.json').read().splitlines()[-1]);print('npt',$npt,d['value'],d['ms_per_step'],d['roofline']['kernel_avg_us'])"
done
export KSG_WIN_NPT=5
timeout -k 10 200 python tools/probe_fixup.py 5000 2048 > gpurun_out/r04a_probe_npt5.txt 2>&1 || exit 1
unset KSG_WIN_NPT
timeout -k 10 300 python tools/cfg4_ab.py --pods 2000 > gpurun_out/r04a_cfg4_ab.json 2> gpurun_out/r04a_cfg4_ab.err || exit 1
head -20 gpurun_out/r04a_cfg4_ab.json
tail -30 gpurun_out/r04a_probe_npt5.txt
