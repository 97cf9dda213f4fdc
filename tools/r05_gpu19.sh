#!/bin/bash
# Round 5: the what-if class path's BalancedAllocation fractions by Markstein's
# correction from a per-node correctly rounded reciprocal (no f64 division per
# pair).  What-if parity (every class-path case, full-size cfg5 1- and 2-rank),
# then cfg5 A/B against libksg_base.so (the build before it), three alternations,
# and the cfg5 SQ pass on the new build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05w}
M=kube-scheduler-simulator-p9_amd/libksg.so
B=kube-scheduler-simulator-p9_amd/libksg_base.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_whatif_gpu.py tests/test_fullsize_gpu.py::test_cfg5_full_size_whatif_step_matches_oracle tests/test_fullsize_gpu.py::test_cfg5_full_size_sharded_2rank_matches_oracle -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
TAG=${TAG}_ab ARMS="mk:KSG_LIB=$M base:KSG_LIB=$B" BENCH="python tools/bench_config.py 5 --cpu-pods 0" FIELDS="d['value'], d.get('ms_per_step')" REPS=3 bash tools/gpu_ab.sh || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS --output-format csv -d gpurun_out/${TAG}_pmcs5 -o run -- python3 tools/bench_config.py 5 --cpu-pods 0 > gpurun_out/${TAG}_pmcs5.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmcs5.log; exit 1; }
python3 tools/pmc_summary.py "$(find gpurun_out/${TAG}_pmcs5 -name "*counter_collection.csv" -print -quit)" > gpurun_out/${TAG}_cfg5_pmc_sq.csv || exit 1
cat gpurun_out/${TAG}_cfg5_pmc_sq.csv
