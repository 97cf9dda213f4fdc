#!/bin/bash
# GPU-box: run the given pytest targets (default: every -m gpu test) under a time
# limit, log to gpurun_out/$TAG.log, print the tail.
TAG=${TAG:-gputest}
LIMIT=${LIMIT:-900}
mkdir -p gpurun_out
export KSG_PROGRESS=gpurun_out/$TAG.progress
timeout -k 10 $LIMIT python -u -m pytest ${@:-tests -m gpu} -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG.log 2>&1
rc=$?
tail -15 gpurun_out/$TAG.log
exit $rc
