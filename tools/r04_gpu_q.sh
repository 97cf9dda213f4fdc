#!/bin/bash
# GPU box: the persistent chain with pod k+1's reads issued during pod k — parity
# (segments incl. no-overlap / lag, full-size cfg4, edge families, preemption),
# stamps with / without, and the cfg4 A/B.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04q}
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_fullsize_gpu.py tests/test_edge_gpu.py tests/test_preempt_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${T}_tests.log | head; tail -2 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
TAG=$T bash tools/r04_gpu_p.sh || exit 1
timeout -k 10 400 python tools/cfg4_ab.py --var KSG_RUN_OVERLAP --pods 2000 > gpurun_out/${T}_cfg4_ab.json 2> gpurun_out/${T}_cfg4_ab.err || { tail -5 gpurun_out/${T}_cfg4_ab.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_cfg4_ab.json'));print('off',d['off']['us_per_pod'],'on',d['on']['us_per_pod'],'equal',d['results_equal'],d['oracle_ok_off'],d['oracle_ok_on'])"
