#!/bin/bash
# Build tools/repro/asan_driver: the library's sources + the driver in one executable, host code under
# AddressSanitizer (-Xarch_host -fsanitize=address), device code as the product's. Build container only.
set -eu
R=$(cd "$(dirname "$0")/../.." && pwd); C=$R/diffusiondrive_amd/csrc; O=$R/tools/repro/_asan
mkdir -p "$O"
F="-O2 -g -std=c++17 -fPIC --offload-arch=gfx950 -I $C -I $R/include -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
NOCONTRACT="decoder.hip train_loss.hip decoder_mk.hip bevproj.hip tfdec_mk.hip elementwise.hip runtime.cpp"
objs=""
for s in conv_gemm.hip conv_x3.hip conv_x5.hip conv_x6.hip elementwise.hip decoder.hip decoder_mk.hip tfdec_mk.hip \
         bevproj.hip value_proj.hip attention.hip stem_pool.hip features.hip train_loss.hip weights.cpp runtime.cpp ops_abi.cpp; do
  extra=""; case " $NOCONTRACT " in *" $s "*) extra="-ffp-contract=off";; esac
  o=$O/$s.o; objs="$objs $o"
  [ "$o" -nt "$C/$s" ] && [ "$o" -nt "$C/common.h" ] || { /opt/rocm/bin/hipcc $F $extra -c "$C/$s" -o "$o" & }
done
wait
/opt/rocm/bin/hipcc $F -c "$R/tools/repro/asan_driver.cpp" -o "$O/asan_driver.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fsanitize=address -fno-gpu-sanitize -o "$R/tools/repro/asan_driver" $objs "$O/asan_driver.o"
echo "built $R/tools/repro/asan_driver"
