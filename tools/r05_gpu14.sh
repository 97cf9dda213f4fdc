#!/bin/bash
# Round 5, final build (kNPos): the whole -m gpu suite, then the cfg4 PMC passes
# (HBM traffic + SQ mix / waves) and kernel-trace stats.  The first failure ends it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r05_full_gpu LIMIT=900 bash tools/gpu_tests.sh || exit 1
bash tools/pmc_config.sh 4 r05 > gpurun_out/r05_pmc4.log 2>&1 || { tail -20 gpurun_out/r05_pmc4.log; exit 1; }
bash tools/prof_config.sh 4 > gpurun_out/r05_cfg4_kernel_stats.csv 2> gpurun_out/r05_kt4.err || { tail -20 gpurun_out/r05_kt4.err; exit 1; }
cat gpurun_out/r05_cfg4_pmc_sq.csv
head -4 gpurun_out/r05_cfg4_kernel_stats.csv
