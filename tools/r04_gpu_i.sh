#!/bin/bash
# GPU box: window parity, then the cfg2 window period over (prior step in the
# replay | in the merges) x (merge blocks | last tile block), with probes; the
# preemption latency at 50k nodes (every pod a full victim search).
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04i}
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_plugin_api_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
for v in "0 0" "0 1"; do
  set -- $v
  export KSG_WIN_PFIX=$1 KSG_WIN_MB=$2
  timeout -k 10 200 python bench.py --extra "" --cpu-baseline 0 --steps 10 --warmup 2 > gpurun_out/${T}_cfg2_pf$1mb$2.json 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/${T}_cfg2_pf$1mb$2.json').read().splitlines()[-1]);print('pfix',$1,'mb',$2,d['value'],d['ms_per_step'],d['roofline']['kernel_avg_us'])"
  timeout -k 10 200 python tools/probe_fixup.py 5000 2048 > gpurun_out/${T}_probe_pf$1mb$2.txt 2>&1 || exit 1
  sed -n 7,17p gpurun_out/${T}_probe_pf$1mb$2.txt
done
unset KSG_WIN_PFIX KSG_WIN_MB
timeout -k 10 500 python tools/bench_preempt.py --nodes 50000 --pods 8 > gpurun_out/${T}_preempt_bench.json 2> gpurun_out/${T}_preempt_bench.err || { tail -5 gpurun_out/${T}_preempt_bench.err; exit 1; }
cat gpurun_out/${T}_preempt_bench.json
timeout -k 10 300 python tools/dropin_probe.py > gpurun_out/${T}_dropin.json 2> gpurun_out/${T}_dropin.err || { tail -5 gpurun_out/${T}_dropin.err; exit 1; }
cat gpurun_out/${T}_dropin.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/${T}_dropin_prof -o run -- python3 tools/dropin_probe.py > gpurun_out/${T}_dropin_prof.log 2>&1 || { tail -5 gpurun_out/${T}_dropin_prof.log; exit 1; }
find gpurun_out/${T}_dropin_prof -name "*stats.csv" | while read f; do echo "== $f"; head -12 "$f"; done
