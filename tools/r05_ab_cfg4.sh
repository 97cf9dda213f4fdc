#!/bin/bash
# cfg4 A/B of persistent-chain switches (tools/cfg4_ab.py: same cluster, results
# checked equal and against the oracle on the first pods).  Each run limited.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r05ab}
for spec in ${SPECS:-KSG_RUN_BT:256,512 KSG_RUN_OVERLAP:0,1}; do
  var=${spec%%:*}; vals=${spec#*:}
  timeout -k 10 400 python tools/cfg4_ab.py --var $var --vals $vals --pods ${PODS:-2000} --check 100 > gpurun_out/${TAG}_${var}.json 2> gpurun_out/${TAG}_${var}.err || { tail -20 gpurun_out/${TAG}_${var}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_${var}.json'));print('$var', d['off']['us_per_pod'], d['on']['us_per_pod'], d['results_equal'], d['oracle_ok_off'], d['oracle_ok_on'])"
done
