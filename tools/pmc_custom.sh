#!/bin/bash
# GPU box: one rocprofv3 --pmc pass (counters in $3, one block's limits respected by
# the caller) over a tools/bench_config.py run; per-kernel means per dispatch to
# gpurun_out/<tag>.csv.  usage: tools/pmc_custom.sh CONFIG TAG "CTR1 CTR2 ..." [bench_config args]
set -o pipefail
C=$1; TAG=$2; CTRS=$3; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 150 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc_$TAG -o run -- python3 tools/bench_config.py $C --cpu-pods 0 "$@" > gpurun_out/pmc_$TAG.log 2>&1 || exit 1
python3 tools/pmc_summary.py "$(find gpurun_out/pmc_$TAG -name "*counter_collection.csv" -print -quit)" > gpurun_out/$TAG.csv || exit 1
head -8 gpurun_out/$TAG.csv
