#!/bin/bash
# GPU box: sequential-queue throughput of cfg1 / cfg3 / cfg4 (BASELINE.json sizes).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_config.py 1 --pods 1000 > gpurun_out/cfg1.json 2> gpurun_out/cfg1.err || exit 1
timeout -k 10 400 python -u tools/bench_config.py 3 --nodes 15000 --pods 2000 > gpurun_out/cfg3.json 2> gpurun_out/cfg3.err || exit 1
timeout -k 10 600 python -u tools/bench_config.py 4 --nodes 50000 --existing 200000 --pods 1000 --cpu-pods 20 > gpurun_out/cfg4.json 2> gpurun_out/cfg4.err || exit 1
cat gpurun_out/cfg1.json gpurun_out/cfg3.json gpurun_out/cfg4.json
