#!/bin/bash
# GPU box: sharded static windows (2/3 ranks on one GPU, gloo host exchange), the
# static window / distributed suites, preemption parity + latency, and the
# window A/B and cfg3 bench line.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04g}
timeout -k 10 600 python -u -m pytest tests/test_distributed.py tests/test_static_window_gpu.py -m gpu -k "${PYTEST_K:-not nothing}" -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_dist.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/${T}_dist.log | tail -40; tail -3 gpurun_out/${T}_dist.log; [ $rc -ne 0 ] && exit $rc
TAG=$T bash tools/r04_gpu_f.sh
