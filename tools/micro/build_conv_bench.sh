#!/bin/bash
# Build the conv microbenchmark against the in-tree libddmi.so (run python -m diffusiondrive_amd.build first).
#   tools/micro/build_conv_bench.sh          -> tools/micro/conv_bench
#   tools/micro/build_conv_bench.sh x5st     -> tools/micro/x5st/conv_bench against libddmi_x5st.so
#     (DDMI_BUILD_VARIANT=x5st python -m diffusiondrive_amd.build first): also prints conv_x5's
#     per-workgroup prologue / K loop / epilogue s_memtime split per shape (x6st: the same for conv_x6)
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
if [ -n "${1:-}" ] && [ "${1:-}" != "x5st" ] && [ "${1:-}" != "x6st" ]; then
  # any other library variant (DDMI_BUILD_VARIANT=$1): the same benchmark against libddmi_$1.so
  V=$1
  mkdir -p "$R/tools/micro/$V"
  /opt/rocm/bin/hipcc -O2 -std=c++17 --offload-arch=gfx950 -I "$R/diffusiondrive_amd/csrc" -I "$R/include" \
    "$R/tools/micro/conv_bench.cpp" -L "$R/diffusiondrive_amd/_variants" -l:libddmi_$V.so \
    -Wl,-rpath,'$ORIGIN/../../../diffusiondrive_amd/_variants' -o "$R/tools/micro/$V/conv_bench"
  exit 0
fi
if [ "${1:-}" = "x5st" ] || [ "${1:-}" = "x6st" ]; then
  V=$1
  mkdir -p "$R/tools/micro/$V"
  /opt/rocm/bin/hipcc -O2 -std=c++17 -D$(echo ${V:0:2} | tr a-z A-Z)_STAMPS --offload-arch=gfx950 -I "$R/diffusiondrive_amd/csrc" \
    -I "$R/include" "$R/tools/micro/conv_bench.cpp" -L "$R/diffusiondrive_amd/_variants" -l:libddmi_$V.so \
    -Wl,-rpath,'$ORIGIN/../../../diffusiondrive_amd/_variants' -o "$R/tools/micro/$V/conv_bench"
  exit 0
fi
/opt/rocm/bin/hipcc -O2 -std=c++17 --offload-arch=gfx950 -I "$R/diffusiondrive_amd/csrc" -I "$R/include" \
  "$R/tools/micro/conv_bench.cpp" -L "$R/diffusiondrive_amd" -lddmi -Wl,-rpath,'$ORIGIN/../../diffusiondrive_amd' \
  -o "$R/tools/micro/conv_bench"
