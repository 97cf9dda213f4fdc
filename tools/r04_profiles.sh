#!/bin/bash
# GPU box: final-build profiles for profiles/ — the headline (cfg2) bench line with its
# kernel-trace summary and HBM-traffic passes, then cfg3 / cfg4 kernel stats, traffic
# and SQ passes.  usage: tools/r04_profiles.sh TAG
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/headline_profile.sh $TAG || exit 1
bash tools/prof_config.sh 4 --nodes 50000 --existing 200000 --pods 1000 > gpurun_out/${TAG}_cfg4_kernel_stats.csv || exit 1
bash tools/prof_config.sh 3 --nodes 15000 --pods 2000 > gpurun_out/${TAG}_cfg3_kernel_stats.csv || exit 1
bash tools/pmc_config.sh 4 $TAG --nodes 50000 --existing 200000 --pods 600 > /dev/null || exit 1
bash tools/pmc_config.sh 3 $TAG --nodes 15000 --pods 2000 > /dev/null || exit 1
echo profiles done
