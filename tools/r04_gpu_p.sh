#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r04p}
for ov in 1 0; do
  KSG_RUN_OVERLAP=$ov timeout -k 10 240 python -u tools/chain_stamps.py --pods 600 > gpurun_out/${T}_stamps_ov$ov.json 2> gpurun_out/${T}_stamps.err || { tail -5 gpurun_out/${T}_stamps.err; exit 1; }
  echo "== overlap $ov"; grep -A 14 "k_chain_run_us_since" gpurun_out/${T}_stamps_ov$ov.json
done
