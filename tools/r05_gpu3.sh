#!/bin/bash
# Round 5: preemption + events parity, the preemption latency bench, then a cfg4
# A/B of the granule poll sleep (libksg.so vs libksg_s2.so).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r05h}
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_preempt_gpu.py tests/test_events_gpu.py tests/test_default_profile_gpu.py tests/test_volume_gpu.py -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
timeout -k 10 600 python tools/bench_preempt.py > gpurun_out/${TAG}_preempt.json 2> gpurun_out/${TAG}_preempt.err || { tail -20 gpurun_out/${TAG}_preempt.err; exit 1; }
cat gpurun_out/${TAG}_preempt.json
TAG=${TAG}_ab ARMS="a:KSG_LIB=kube-scheduler-simulator-p9_amd/libksg.so b:KSG_LIB=kube-scheduler-simulator-p9_amd/libksg_s2.so" BENCH="python bench.py --extra 4 --cpu-baseline 0 --steps 5 --warmup 1" FIELDS="d['value'], d['cfg4']['us_per_pod']" REPS=2 bash tools/gpu_ab.sh
