#!/bin/bash
# GPU box: what-if record kernels — parity subset, then kernel-trace stats of the
# cfg5 bench with and without an A/B switch (env $1, default KSG_WHATIF_NOHOT).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
SW=${1:-KSG_WHATIF_NOHOT}
timeout -k 10 300 python3 -u -m pytest tests/test_whatif_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "cfg5 or records" > gpurun_out/wi_ab_test.log 2>&1 || exit 1
for v in a b; do
  if [ $v = b ]; then export $SW=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wi_ab_$v -o run -- python3 bench_whatif.py --cpu-pods 0 --steps 2 > gpurun_out/wi_ab_$v.log 2>&1 || exit 1
  cp "$(find gpurun_out/wi_ab_$v -name "*kernel_stats.csv" -print -quit)" gpurun_out/wi_ab_${v}_kstats.csv || exit 1
done
