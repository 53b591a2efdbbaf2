#!/bin/bash
# Decoder / tf-decoder megakernel diagnostics: per-phase stamps (stamps library) at B = 64 and B = 1, and a kernel
# trace of batch-1 forwards on the default handle. Needs diffusiondrive_amd/_variants/libddmi_stamps.so (built on
# the CPU: DDMI_BUILD_VARIANT=stamps python -m diffusiondrive_amd.build) and _variants not in .gpurunignore.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; T=${1:-diag}
for b in 64 1; do
  timeout -k 10 200 env DDMI_STAMP_B=$b python -u tools/debug/mk_stamps.py > gpurun_out/${T}_mk_b$b.log 2>&1
  rc=$?; echo "[mk B=$b] rc=$rc"; cat gpurun_out/${T}_mk_b$b.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 env DDMI_STAMP_B=$b python -u tools/debug/tf_stamps.py > gpurun_out/${T}_tf_b$b.log 2>&1
  rc=$?; echo "[tf B=$b] rc=$rc"; cat gpurun_out/${T}_tf_b$b.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${T}_b1trace" -- python3 "$R/tools/micro/b1_trace.py" > "$R/gpurun_out/${T}_b1trace.log" 2>&1
rc=$?; echo "[b1 trace] rc=$rc"; grep b1_trace "$R/gpurun_out/${T}_b1trace.log"; exit $rc
