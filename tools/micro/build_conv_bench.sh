#!/bin/bash
# Build the conv microbenchmark against the in-tree libddmi.so (run python -m diffusiondrive_amd.build first).
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
/opt/rocm/bin/hipcc -O2 -std=c++17 --offload-arch=gfx950 -I "$R/diffusiondrive_amd/csrc" -I "$R/include" \
  "$R/tools/micro/conv_bench.cpp" -L "$R/diffusiondrive_amd" -lddmi -Wl,-rpath,'$ORIGIN/../../diffusiondrive_amd' \
  -o "$R/tools/micro/conv_bench"
