set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_whatif_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "cfg5 or records" > gpurun_out/wi_ab_test.log 2>&1 || exit 1
for w in 6 8; do
  KSG_WI_REC1_WAVES=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wi_ab$w -o run -- python3 bench_whatif.py --cpu-pods 0 --steps 2 > gpurun_out/wi_ab$w.log 2>&1 || exit 1
  cp "$(find gpurun_out/wi_ab$w -name "*kernel_stats.csv" -print -quit)" gpurun_out/wi_ab${w}_kstats.csv || exit 1
done
