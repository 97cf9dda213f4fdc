#!/bin/bash
# Builds libksg.so (HIP engine + C++ host layer) in-tree for gfx950.
set -e
cd "$(dirname "$0")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
  -Wno-unused-result -o libksg.so csrc/engine.hip csrc/host.cpp csrc/synth.cpp -L/opt/rocm/lib -lrccl "$@"
