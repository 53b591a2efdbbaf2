#!/bin/bash
# GPU box: kernel traces of the two-stream bench graph with the decoder megakernel on and off (A/B of the
# trajectory-head critical path; read with tools/tail_view.py). Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for mk in 1 0; do
  DDMI_DECODER_MK=$mk timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/tl_mk$mk" -o run -- python "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-compare > "$R/gpurun_out/tl_mk$mk.log" 2>&1
  rc=$?; echo "[trace mk=$mk] rc=$rc"; grep '^{' "$R/gpurun_out/tl_mk$mk.log" | cut -c1-200; [ $rc -ne 0 ] && exit $rc
done
exit 0
