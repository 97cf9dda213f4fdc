#!/bin/bash
# Round 5: the drop-in cycle's device work.  k_pc_build counts few-domain slots
# (and pc_tot) per 1,024-row block in LDS (KSG_PC_AGG); k_view sizes the
# PodTopologySpread / InterPodAffinity raw rows by the summary's range
# (KSG_VIEW_NARROW).  Class-table / view parity, then the C-ABI drop-in latency
# at cfg4 per arm (three alternations), cfg2 once, and kernel traces per arm.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05t}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cycle_gpu.py tests/test_plugin_api_gpu.py tests/test_events_gpu.py tests/test_parity_gpu.py tests/test_fullsize_gpu.py::test_cfg4_full_size_matches_oracle -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
arm() { case $1 in new) echo "KSG_PC_AGG=1 KSG_VIEW_NARROW=1";; agg) echo "KSG_PC_AGG=1 KSG_VIEW_NARROW=0";; old) echo "KSG_PC_AGG=0 KSG_VIEW_NARROW=0";; esac; }
for r in 1 2 3; do
  for a in new agg old; do
    env $(arm $a) timeout -k 10 300 python tools/dropin_c.py --cfg 4 --out gpurun_out/${TAG}_dropin_$a.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin.err || { tail -20 gpurun_out/${TAG}_dropin.err; exit 1; }
  done
done
timeout -k 10 300 python tools/dropin_c.py --cfg 2 --out gpurun_out/${TAG}_dropin_cfg2.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin.err || { tail -20 gpurun_out/${TAG}_dropin.err; exit 1; }
for a in new old; do
  export $(arm $a)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_$a -o run -- python3 tools/dropin_c.py --cfg 4 --count 100 > gpurun_out/${TAG}_kt_$a.log 2>&1 || { tail -20 gpurun_out/${TAG}_kt_$a.log; exit 1; }
done
for a in new agg old; do echo "== $a"; cut -c1-120 gpurun_out/${TAG}_dropin_$a.jsonl; done
