#!/bin/bash
# GPU box A/B runner (replaces round 4's one-off tools/r04_gpu_*.sh recipes).
#
#   TAG=r05x ARMS="a:KSG_LIB=kube-scheduler-simulator-p9_amd/libksg.so b:KSG_LIB=kube-scheduler-simulator-p9_amd/libksg_b.so" \
#   BENCH="python bench.py --extra '' --cpu-baseline 0 --steps 10 --warmup 2" REPS=2 \
#   PARITY="tests/test_parity_gpu.py -k cfg2_large" PARITY_ARM=b bash tools/gpu_ab.sh
#
# ARMS   space-separated "name:VAR=value[,VAR=value...]" (the environment of each arm;
#        KSG_LIB picks a library build, KSG_* switches pick an engine path)
# BENCH  the command timed per arm (its last stdout line is the JSON it reports)
# FIELDS python expression over the JSON `d` printed per run (default: value, kernel µs)
# REPS   alternations of the arms (default 2)
# PARITY pytest arguments run once per arm named in PARITY_ARM (default: every arm), first
# Every GPU step runs under its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-ab}
REPS=${REPS:-2}
BENCH=${BENCH:-python bench.py --extra '' --cpu-baseline 0 --steps 10 --warmup 2}
FIELDS=${FIELDS:-"d['value'], d['roofline']['kernel_avg_us']"}
arm_env() {  # "name:A=1,B=2" -> "A=1 B=2"
  echo "${1#*:}" | tr ',' ' '
}
if [ -n "$PARITY" ]; then
  for arm in $ARMS; do
    name=${arm%%:*}
    case " ${PARITY_ARM:-$name} " in *" $name "*) ;; *) continue ;; esac
    env $(arm_env "$arm") timeout -k 10 ${PARITY_LIMIT:-600} python -u -m pytest -x -q --timeout 300 --timeout-method thread $PARITY \
      > gpurun_out/${TAG}_parity_${name}.log 2>&1 || { tail -30 gpurun_out/${TAG}_parity_${name}.log; exit 1; }
    echo "parity $name: $(tail -1 gpurun_out/${TAG}_parity_${name}.log)"
  done
fi
[ -z "$BENCH" ] && exit 0
for rep in $(seq 1 $REPS); do
  for arm in $ARMS; do
    name=${arm%%:*}
    out=gpurun_out/${TAG}_${name}_${rep}.json
    env $(arm_env "$arm") timeout -k 10 ${BENCH_LIMIT:-300} bash -c "$BENCH" > $out 2> ${out%.json}.err || { tail -20 ${out%.json}.err; exit 1; }
    python -c "import json;d=json.loads(open('$out').read().splitlines()[-1]);print('$name', $rep, $FIELDS)"
  done
done
