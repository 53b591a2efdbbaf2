#!/bin/bash
# GPU box: bench A/B of the tf-decoder megakernel (on / off / on) and a two-stream kernel trace with it on
# (read with tools/tail_view.py). Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
NOTESTS=1 bash tools/gpu_ab.sh "DDMI_TFDEC_MK=1" "DDMI_TFDEC_MK=0" "DDMI_TFDEC_MK=1" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/tl_tf" -o run -- python "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-compare > "$R/gpurun_out/tl_tf.log" 2>&1
rc=$?; echo "[trace] rc=$rc"; exit $rc
