#!/bin/bash
# GPU box: cfg5 what-if (bench_whatif.py, 2 steps) — kernel-trace stats, then
# PMC passes one counter group per run: HBM bytes (FETCH_SIZE, WRITE_SIZE), the
# SQ instruction mix and an LDS / wait pass.  usage: tools/pmc_whatif.sh TAG
set -o pipefail
TAG=${1:-r03}
export TMPDIR=/tmp
mkdir -p gpurun_out
A="--steps 2 --warmup 1 --cpu-pods 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wi_kt -o run -- python3 bench_whatif.py $A > gpurun_out/wi_kt.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/wi_f -o run -- python3 bench_whatif.py $A > gpurun_out/wi_f.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/wi_w -o run -- python3 bench_whatif.py $A > gpurun_out/wi_w.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/wi_f gpurun_out/wi_w "cfg5:" > gpurun_out/${TAG}_cfg5_pmc_traffic.json || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/wi_s -o run -- python3 bench_whatif.py $A > gpurun_out/wi_s.log 2>&1 || exit 1
python3 tools/pmc_summary.py "$(find gpurun_out/wi_s -name "*counter_collection.csv" -print -quit)" > gpurun_out/${TAG}_cfg5_pmc_sq.csv || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/wi_l -o run -- python3 bench_whatif.py $A > gpurun_out/wi_l.log 2>&1 || exit 1
python3 tools/pmc_summary.py "$(find gpurun_out/wi_l -name "*counter_collection.csv" -print -quit)" > gpurun_out/${TAG}_cfg5_pmc_lds.csv || exit 1
find gpurun_out/wi_kt -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_cfg5_kernel_stats.csv \;
head -6 gpurun_out/${TAG}_cfg5_kernel_stats.csv
cat gpurun_out/${TAG}_cfg5_pmc_sq.csv gpurun_out/${TAG}_cfg5_pmc_lds.csv
grep -A8 k_whatif gpurun_out/${TAG}_cfg5_pmc_traffic.json | head -30
