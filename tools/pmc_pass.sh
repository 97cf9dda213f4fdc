#!/bin/bash
# On the GPU box: kernel-trace stats + two PMC passes (FETCH_SIZE, WRITE_SIZE)
# over short bench runs; summaries land in gpurun_out/ (copy to profiles/).
set -o pipefail
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd "$ROOT" || exit 1
mkdir -p gpurun_out
ARGS="--steps 2 --warmup 1 --cpu-baseline 0"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktrace -o run -- python3 bench.py $ARGS > gpurun_out/ktrace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py $ARGS > gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py $ARGS > gpurun_out/pmc_write.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/${TAG}_pmc_traffic.json || exit 1
find gpurun_out/ktrace -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
cat gpurun_out/${TAG}_pmc_traffic.json
head -5 gpurun_out/${TAG}_kernel_stats.csv
