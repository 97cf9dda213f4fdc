#!/bin/bash
# Round 5 final build, part B: per-config PMC passes (HBM traffic + SQ instruction
# mix / waves) for cfg3 and cfg4, the cfg5 what-if passes, kernel-trace stats of
# cfg3 / cfg4, and cfg4 block-0 stamps.  Each step limited; the first failure ends it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cycle_gpu.py tests/test_events_gpu.py tests/test_plugin_api_gpu.py -m gpu > gpurun_out/r05_final_b_gputest.log 2>&1 || { tail -30 gpurun_out/r05_final_b_gputest.log; exit 1; }
tail -1 gpurun_out/r05_final_b_gputest.log
bash tools/pmc_config.sh 3 r05 > gpurun_out/r05_pmc3.log 2>&1 || { tail -20 gpurun_out/r05_pmc3.log; exit 1; }
bash tools/pmc_config.sh 4 r05 > gpurun_out/r05_pmc4.log 2>&1 || { tail -20 gpurun_out/r05_pmc4.log; exit 1; }
bash tools/prof_config.sh 3 > gpurun_out/r05_cfg3_kernel_stats.csv 2> gpurun_out/r05_kt3.err || { tail -20 gpurun_out/r05_kt3.err; exit 1; }
bash tools/prof_config.sh 4 > gpurun_out/r05_cfg4_kernel_stats.csv 2> gpurun_out/r05_kt4.err || { tail -20 gpurun_out/r05_kt4.err; exit 1; }
bash tools/pmc_whatif.sh r05 > gpurun_out/r05_wi.log 2>&1 || { tail -20 gpurun_out/r05_wi.log; exit 1; }
timeout -k 10 300 python tools/chain_stamps.py --pods 1200 > gpurun_out/r05_final_stamps.json 2> gpurun_out/r05_final_stamps.err || { tail -20 gpurun_out/r05_final_stamps.err; exit 1; }
cat gpurun_out/r05_cfg3_pmc_sq.csv gpurun_out/r05_cfg4_pmc_sq.csv
head -4 gpurun_out/r05_cfg3_kernel_stats.csv gpurun_out/r05_cfg4_kernel_stats.csv
