#!/bin/bash
# Round 5: per-position loops bounded by the kernel's plugin set (kNPos) — the
# persistent chain's parity and a cfg4 A/B against libksg_base.so (HEAD before it).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05u}
M=kube-scheduler-simulator-p9_amd/libksg.so
B=kube-scheduler-simulator-p9_amd/libksg_base.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_parity_gpu.py tests/test_fullsize_gpu.py::test_cfg4_full_size_matches_oracle tests/test_edge_gpu.py -m gpu > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
TAG=${TAG}_ab ARMS="npos:KSG_LIB=$M base:KSG_LIB=$B" BENCH="python bench.py --extra 4 --cpu-baseline 0 --steps 5 --warmup 1" FIELDS="d['cfg4']['us_per_pod'], d['cfg4']['roofline']['kernel_avg_us']" REPS=3 bash tools/gpu_ab.sh
# then the final bench line and the headline's kernel trace / PMC passes on this build
bash tools/r05_final_a.sh
