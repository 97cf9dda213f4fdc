#!/bin/bash
# Round 5: cfg5 what-if step (bench_whatif.py) A/B — BalancedAllocation fractions
# by Markstein's correction (libksg.so) against the build before it
# (libksg_base.so), three alternations — then the SQ pass and kernel stats of the
# new build.  (Parity: r05_gpu19.sh, whatif + full-size cfg5 tests.)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05x}
M=kube-scheduler-simulator-p9_amd/libksg.so
B=kube-scheduler-simulator-p9_amd/libksg_base.so
TAG=${TAG}_ab ARMS="mk:KSG_LIB=$M base:KSG_LIB=$B" BENCH="python bench_whatif.py --steps 4 --warmup 1 --cpu-pods 0" FIELDS="d['value'], d.get('ms_per_step')" REPS=3 bash tools/gpu_ab.sh || exit 1
A="--steps 2 --warmup 1 --cpu-pods 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_wi_kt -o run -- python3 bench_whatif.py $A > gpurun_out/${TAG}_wi_kt.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_wi_s -o run -- python3 bench_whatif.py $A > gpurun_out/${TAG}_wi_s.log 2>&1 || exit 1
python3 tools/pmc_summary.py "$(find gpurun_out/${TAG}_wi_s -name "*counter_collection.csv" -print -quit)" > gpurun_out/${TAG}_cfg5_pmc_sq.csv || exit 1
find gpurun_out/${TAG}_wi_kt -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_cfg5_kernel_stats.csv \;
head -4 gpurun_out/${TAG}_cfg5_kernel_stats.csv | cut -c1-200
cat gpurun_out/${TAG}_cfg5_pmc_sq.csv
