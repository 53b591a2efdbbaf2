#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  DDMI_GEMM_LAT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/gm$v" -o run -- python3 "$R/tools/micro/gemm_bench.py" > "$R/gpurun_out/gm$v.log" 2>&1
  rc=$?; echo "[lat=$v] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
