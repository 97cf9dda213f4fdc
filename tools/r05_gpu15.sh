#!/bin/bash
# Round 5: the drop-in cycle's class step.  k_pc_build reads the new classes'
# requirement-key label columns up front (KSG_PC_PREFETCH) and the cycle's
# program goes out in the class upload (KSG_PLACE_FUSED).  Class-table parity
# (cycle / plugin API / events / cfg2-cfg4 parity), then the C-ABI drop-in
# latency at cfg4 per arm (two alternations) and kernel traces of the drop-in run.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05s}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cycle_gpu.py tests/test_plugin_api_gpu.py tests/test_events_gpu.py tests/test_parity_gpu.py -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
arm() { case $1 in base) echo "KSG_PC_PREFETCH=0 KSG_PLACE_FUSED=0";; pf) echo "KSG_PC_PREFETCH=1 KSG_PLACE_FUSED=0";; both) echo "KSG_PC_PREFETCH=1 KSG_PLACE_FUSED=1";; esac; }
for r in 1 2; do
  for a in both pf base; do
    env $(arm $a) timeout -k 10 300 python tools/dropin_c.py --cfg 4 --out gpurun_out/${TAG}_dropin_$a.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin.err || { tail -20 gpurun_out/${TAG}_dropin.err; exit 1; }
  done
done
timeout -k 10 300 python tools/dropin_c.py --cfg 2 --out gpurun_out/${TAG}_dropin_cfg2.jsonl > /dev/null 2> gpurun_out/${TAG}_dropin.err || { tail -20 gpurun_out/${TAG}_dropin.err; exit 1; }
for a in both base; do
  export $(arm $a)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_$a -o run -- python3 tools/dropin_c.py --cfg 4 --count 100 > gpurun_out/${TAG}_kt_$a.log 2>&1 || { tail -20 gpurun_out/${TAG}_kt_$a.log; exit 1; }
done
for a in both pf base; do echo "== $a"; cut -c1-330 gpurun_out/${TAG}_dropin_$a.jsonl; done
cut -c1-200 gpurun_out/${TAG}_dropin_cfg2.jsonl
for a in both base; do echo "== kt $a"; find gpurun_out/${TAG}_kt_$a -name "*kernel_stats.csv" -exec cut -c1-40,100-200 {} \; | head -12; done
