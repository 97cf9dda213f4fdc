#!/bin/bash
# GPU box, a round's final build: the profiles/ evidence -- the headline's kernel
# trace and HBM-traffic PMC passes (headline_profile.sh), per-config PMC passes
# (traffic + SQ instruction mix) for cfg3 / cfg4, the cfg5 what-if passes,
# kernel-trace stats of cfg3 / cfg4 and the cfg4 block-0 stamps.
#   bash tools/final_profiles.sh r06
# Results under gpurun_out/ (copy what is cited to profiles/).  Each step limited;
# the first failure ends it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${1:-r06}
bash tools/headline_profile.sh $R > gpurun_out/${R}_headline.log 2>&1 || { tail -20 gpurun_out/${R}_headline.log; exit 1; }
bash tools/pmc_config.sh 3 $R > gpurun_out/${R}_pmc3.log 2>&1 || { tail -20 gpurun_out/${R}_pmc3.log; exit 1; }
bash tools/pmc_config.sh 4 $R > gpurun_out/${R}_pmc4.log 2>&1 || { tail -20 gpurun_out/${R}_pmc4.log; exit 1; }
bash tools/prof_config.sh 3 > gpurun_out/${R}_cfg3_kernel_stats.csv 2> gpurun_out/${R}_kt3.err || { tail -20 gpurun_out/${R}_kt3.err; exit 1; }
bash tools/prof_config.sh 4 > gpurun_out/${R}_cfg4_kernel_stats.csv 2> gpurun_out/${R}_kt4.err || { tail -20 gpurun_out/${R}_kt4.err; exit 1; }
bash tools/pmc_whatif.sh $R > gpurun_out/${R}_wi.log 2>&1 || { tail -20 gpurun_out/${R}_wi.log; exit 1; }
timeout -k 10 300 python tools/chain_stamps.py --pods 1200 > gpurun_out/${R}_final_stamps.json 2> gpurun_out/${R}_final_stamps.err || { tail -20 gpurun_out/${R}_final_stamps.err; exit 1; }
cat gpurun_out/${R}_cfg3_pmc_sq.csv gpurun_out/${R}_cfg4_pmc_sq.csv
head -4 gpurun_out/${R}_cfg3_kernel_stats.csv gpurun_out/${R}_cfg4_kernel_stats.csv
