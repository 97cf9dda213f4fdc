#!/bin/bash
# GPU-box check: parity tests, then the benchmark (each step under its own time limit).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?
tail -5 gpurun_out/gputest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python bench.py ${BENCH_ARGS:---cpu-baseline 0} > gpurun_out/bench.log 2>&1
rc=$?
tail -3 gpurun_out/bench.log
exit $rc
