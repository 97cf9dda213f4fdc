#!/bin/bash
# GPU box: the headline bench line, its rocprofv3 kernel-trace summary and the
# HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs), for profiles/.
# usage: tools/headline_profile.sh TAG
set -o pipefail
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
B="--extra= --cpu-baseline 0 --steps 3"
timeout -k 10 420 python3 -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
echo "bench done"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 bench.py $B > gpurun_out/${TAG}_kt.log 2>&1 || exit 1
cp "$(find gpurun_out/${TAG}_kt -name "*kernel_stats.csv" -print -quit)" gpurun_out/${TAG}_cfg2_kernel_stats.csv || exit 1
echo "kernel trace done"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pf -o run -- python3 bench.py $B > gpurun_out/${TAG}_pf.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pw -o run -- python3 bench.py $B > gpurun_out/${TAG}_pw.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/${TAG}_pf gpurun_out/${TAG}_pw "" > gpurun_out/${TAG}_cfg2_pmc_traffic.json || exit 1
echo "pmc done"
head -c 400 gpurun_out/${TAG}_bench.json
