#!/bin/bash
# GPU box: PMC passes over one config run (tools/bench_config.py), one counter group per
# run: FETCH_SIZE, WRITE_SIZE (-> HBM bytes per dispatch, keys "cfgC:<kernel>") and an SQ
# pass (VALU instructions, waves, busy cycles).  usage: tools/pmc_config.sh C TAG [bench_config args]
set -o pipefail
C=$1; TAG=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
A="$C --cpu-pods 0 $*"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_cfg$C -o run -- python3 tools/bench_config.py $A > gpurun_out/pmcf_cfg$C.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_cfg$C -o run -- python3 tools/bench_config.py $A > gpurun_out/pmcw_cfg$C.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/pmcf_cfg$C gpurun_out/pmcw_cfg$C "cfg$C:" > gpurun_out/${TAG}_cfg${C}_pmc_traffic.json || exit 1
# persistent segments: per pod cycle too (the bench line's k_chain_run "launch" is one pod)
python3 - gpurun_out/${TAG}_cfg${C}_pmc_traffic.json gpurun_out/pmcf_cfg$C.log "cfg$C:k_chain_run" <<'PY' || exit 1
import json, sys
f, log, key = sys.argv[1:4]
d = json.load(open(f))
k = d["kernels"].get(key)
line = [l for l in open(log) if l.startswith("{")]
if k and line:
    pods, segs = json.loads(line[-1]).get("run_counts", [0, 0])
    if segs:
        k["pods_per_dispatch"] = pods / segs
        k["hbm_bytes_per_pod"] = k["hbm_bytes_per_dispatch"] / k["pods_per_dispatch"]
        json.dump(d, open(f, "w"), indent=1)
PY
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS --output-format csv -d gpurun_out/pmcs_cfg$C -o run -- python3 tools/bench_config.py $A > gpurun_out/pmcs_cfg$C.log 2>&1 || exit 1
python3 tools/pmc_summary.py "$(find gpurun_out/pmcs_cfg$C -name "*counter_collection.csv" -print -quit)" > gpurun_out/${TAG}_cfg${C}_pmc_sq.csv || exit 1
cat gpurun_out/${TAG}_cfg${C}_pmc_traffic.json
