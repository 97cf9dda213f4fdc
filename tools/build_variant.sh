#!/bin/bash
# A variant build of libksg.so for A/B runs: engine.hip with extra compiler flags
# into build_<name>/, linked with the main build's host and synth objects, as
# kube-scheduler-simulator-p9_amd/libksg_<name>.so (pick it with KSG_LIB=...).
#   tools/build_variant.sh NAME "-DKSG_RUN_SLEEP=2 ..."
set -e
cd "$(dirname "$0")/../kube-scheduler-simulator-p9_amd"
name=$1; shift
mkdir -p build_$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result $* -c -o build_$name/engine.o csrc/engine.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o libksg_$name.so build_$name/engine.o build/host.o build/synth.o -L/opt/rocm/lib -lrccl
