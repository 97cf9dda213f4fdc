#!/bin/bash
# GPU box: kernel-trace stats of one config run (tools/bench_config.py), summary to gpurun_out/
set -o pipefail
C=${1:-3}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_cfg$C -o run -- python3 tools/bench_config.py $C --cpu-pods 0 "$@" > gpurun_out/kt_cfg$C.log 2>&1 || exit 1
find gpurun_out/kt_cfg$C -name "*kernel_stats.csv" -exec cat {} \;
