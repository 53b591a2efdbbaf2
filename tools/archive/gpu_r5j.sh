#!/bin/bash
# round 5j: where the union value_proj's time goes - DDMI_VPROJ_DIAG (bit 0: union loads read nothing, bit 1: B DMAs
# read nothing; timing only) on the bench workload, one forward at a time, profiled per-class device time
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for d in 0 1 2 3 0; do
  DDMI_VPROJ_DIAG=$d timeout -k 10 200 python bench.py --in-flight 1 --no-cpu-baseline --no-compare --steps 20 > gpurun_out/r5j.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc [diag $d]"; tail -5 gpurun_out/r5j.log; exit $rc; }
  echo "[vproj diag $d] $(tail -1 gpurun_out/r5j.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["device_ms_per_step"]["value_proj"], d["decoder_cross_attention"]["avg_launch_ms"])')"
done | tee gpurun_out/r5j_vproj_diag.txt
