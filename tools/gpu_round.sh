#!/bin/bash
# GPU-box session: parity tests (full-size ones report progress to a file), then
# the benchmark; each step under its own time limit, stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export KSG_PROGRESS=gpurun_out/progress.log
timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest ${TEST_ARGS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?
tail -5 gpurun_out/gputest.log
[ $rc -ne 0 ] && exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?
tail -3 gpurun_out/bench.log
exit $rc
