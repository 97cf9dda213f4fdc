#!/bin/bash
# GPU box: current-build profiles of cfg3 / cfg4 (kernel stats, PMC traffic + SQ) and
# the cfg4 chain stamps, all under gpurun_out/ with the given tag.
set -o pipefail
TAG=${1:-r03}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/chain_stamps.py --pods 600 > gpurun_out/${TAG}_cfg4_chain_stamps.json 2> gpurun_out/stamps.err || exit 1
bash tools/prof_config.sh 4 --nodes 50000 --existing 200000 --pods 1000 > gpurun_out/${TAG}_cfg4_kernel_stats.csv || exit 1
bash tools/prof_config.sh 3 --nodes 15000 --pods 2000 > gpurun_out/${TAG}_cfg3_kernel_stats.csv || exit 1
bash tools/pmc_config.sh 4 $TAG --nodes 50000 --existing 200000 --pods 600 > /dev/null || exit 1
bash tools/pmc_config.sh 3 $TAG --nodes 15000 --pods 2000 > /dev/null || exit 1
echo done
