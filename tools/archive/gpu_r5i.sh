#!/bin/bash
# round 5i: A/B of the decoder query groups and the union value_proj split at B = 64, one forward at a time and at
# 3 in flight (same box, alternating)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "X=0" "DDMI_MK_GROUPS=2" "DDMI_MK_GROUPS=4" "DDMI_VPROJ_USPLIT=2"; do
    env $cfg timeout -k 10 200 python bench.py --in-flight 1 --no-cpu-baseline --no-compare --steps 60 > gpurun_out/r5i_if1.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc [$cfg]"; tail -5 gpurun_out/r5i_if1.log; exit $rc; }
    echo "[if1 $cfg] $(tail -1 gpurun_out/r5i_if1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["device_ms_per_step"]["decoder"], d["device_ms_per_step"]["value_proj"])')"
  done
done | tee gpurun_out/r5i_ab.txt
for cfg in "X=0" "DDMI_MK_GROUPS=2" "X=0" "DDMI_MK_GROUPS=2"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --steps 100 > gpurun_out/r5i_if3.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc [$cfg]"; tail -5 gpurun_out/r5i_if3.log; exit $rc; }
  echo "[if3 $cfg] $(tail -1 gpurun_out/r5i_if3.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
done | tee -a gpurun_out/r5i_ab.txt
