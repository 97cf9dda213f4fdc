#!/bin/bash
# Builds libksg.so (HIP engine + C++ host layer) in-tree for gfx950: the three
# translation units in parallel, each rebuilt only when it or a header changed.
# Extra compiler flags go in EXTRA="..." (a change of flags needs `make clean`).
set -e
cd "$(dirname "$0")"
make -s -j3 libksg.so EXTRA="$*"
