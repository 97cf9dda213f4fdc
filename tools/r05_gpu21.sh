#!/bin/bash
# Round 5: k_final specialised for the Fit/BA/PTS/IPA plugin set (kNPos bounds;
# KSG_FINAL_PM).  Table-chain parity (cycle / plugin API / parity incl. cfg4),
# then the C-ABI drop-in at cfg4 per arm, three alternations.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05y}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cycle_gpu.py tests/test_plugin_api_gpu.py tests/test_parity_gpu.py tests/test_default_profile_gpu.py -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
for r in 1 2 3; do
  for a in 1 0; do
    KSG_FINAL_PM=$a timeout -k 10 300 python tools/dropin_c.py --cfg 4 --out gpurun_out/${TAG}_dropin_pm$a.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin.err || { tail -20 gpurun_out/${TAG}_dropin.err; exit 1; }
  done
done
export KSG_FINAL_PM=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 tools/dropin_c.py --cfg 4 --count 100 > gpurun_out/${TAG}_kt.log 2>&1 || { tail -20 gpurun_out/${TAG}_kt.log; exit 1; }
for a in 1 0; do echo "== pm$a"; cut -c1-120 gpurun_out/${TAG}_dropin_pm$a.jsonl; done
grep -h "k_final\|k_eval" $(find gpurun_out/${TAG}_kt -name "*kernel_stats.csv") | cut -c1-60,100-200
