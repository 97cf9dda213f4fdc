#!/bin/bash
# GPU box: the persistent chain with pod overlap — parity (segments, full-size cfg4,
# edge families), then the cfg4 A/B of KSG_RUN_OVERLAP.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04o}
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_fullsize_gpu.py tests/test_edge_gpu.py tests/test_preempt_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${T}_tests.log | head; tail -2 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/cfg4_ab.py --var KSG_RUN_OVERLAP --pods 2000 > gpurun_out/${T}_cfg4_ab.json 2> gpurun_out/${T}_cfg4_ab.err || { tail -5 gpurun_out/${T}_cfg4_ab.err; exit 1; }
cat gpurun_out/${T}_cfg4_ab.json
