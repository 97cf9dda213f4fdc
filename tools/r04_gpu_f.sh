#!/bin/bash
# GPU box: preemption parity (batched and per-node searches) and latency at 50k
# nodes; the window A/B (merge blocks) and the cfg3 line with its k_static split.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04f}
timeout -k 10 300 python -u -m pytest tests/test_preempt_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_preempt.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_preempt.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/bench_preempt.py --nodes 50000 --pods 8 > gpurun_out/${T}_preempt_bench.json 2> gpurun_out/${T}_preempt_bench.err || { tail -5 gpurun_out/${T}_preempt_bench.err; exit 1; }
cat gpurun_out/${T}_preempt_bench.json
TAG=$T bash tools/r04_gpu_b.sh || exit 1
timeout -k 10 300 python bench.py --extra 3 --cpu-baseline 0 --steps 5 > gpurun_out/${T}_bench3.json 2> gpurun_out/${T}_bench3.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/${T}_bench3.json').read().splitlines()[-1]);print(json.dumps(d['cfg3']['roofline'])[:900])"
