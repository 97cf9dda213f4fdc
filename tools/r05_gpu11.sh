#!/bin/bash
# Round 5: static records beside the loop launched first on the idle CUs
# (k_static_dec_run) and status bytes in the granules' spare bits — parity of the
# static windows and the persistent chain, a PMC pass over cfg3 (kernels one at a
# time: the case that deadlocked the verdict-first launch), then A/Bs: cfg3 with
# and without the overlap, cfg4 against libksg_base.so (the previous build).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05s}
M=kube-scheduler-simulator-p9_amd/libksg.so
B=kube-scheduler-simulator-p9_amd/libksg_base.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_static_window_gpu.py tests/test_parity_gpu.py tests/test_fullsize_gpu.py::test_cfg4_full_size_matches_oracle -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmcf3 -o run -- python3 tools/bench_config.py 3 --cpu-pods 0 > gpurun_out/${TAG}_pmcf3.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmcf3.log; exit 1; }
grep -h "^{" gpurun_out/${TAG}_pmcf3.log | tail -1 | cut -c1-300 || true
TAG=${TAG}_c3 ARMS="overlap:KSG_LIB=$M before:KSG_LIB=$M,KSG_STATIC_OVERLAP=0" BENCH="python bench.py --extra 3 --cpu-baseline 0 --steps 10 --warmup 2" FIELDS="d['cfg3']['value'], d['cfg3']['roofline']['kernel_avg_us']" REPS=2 bash tools/gpu_ab.sh || exit 1
TAG=${TAG}_c4 ARMS="spare:KSG_LIB=$M base:KSG_LIB=$B" BENCH="python bench.py --extra 4 --cpu-baseline 0 --steps 5 --warmup 1" FIELDS="d['cfg4']['us_per_pod'], d['cfg4']['roofline']['kernel_avg_us']" REPS=3 bash tools/gpu_ab.sh
