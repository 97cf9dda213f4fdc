#!/bin/bash
# GPU box: cfg4 A/B of Fit/BA after the class-table reads are issued (B, libksg.so)
# vs before (A, libksg_a.so), both orders, then the persistent-chain parity tests.
set -o pipefail
mkdir -p gpurun_out
A=kube-scheduler-simulator-p9_amd/libksg_a.so
B=kube-scheduler-simulator-p9_amd/libksg.so
timeout -k 10 300 python -u tools/cfg4_ab.py --var KSG_LIB --vals $A,$B --pods 3000 --check 100 > gpurun_out/r04r_ab1.json 2>&1 || { tail -5 gpurun_out/r04r_ab1.json; exit 1; }
timeout -k 10 300 python -u tools/cfg4_ab.py --var KSG_LIB --vals $B,$A --pods 3000 --check 100 > gpurun_out/r04r_ab2.json 2>&1 || { tail -5 gpurun_out/r04r_ab2.json; exit 1; }
grep -h "us_per_pod\|equal\|oracle_ok" gpurun_out/r04r_ab1.json gpurun_out/r04r_ab2.json
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k "persistent" > gpurun_out/r04r_parity.log 2>&1; rc=$?
tail -3 gpurun_out/r04r_parity.log
exit $rc
