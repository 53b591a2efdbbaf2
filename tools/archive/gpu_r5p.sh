#!/bin/bash
# round 5p: one B = 64 forward at a time (default two-stream handle), decoder query groups 1 vs 2, 200 steps, alternating
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for rep in 1 2 3 4; do
  for cfg in "X=0" "DDMI_MK_GROUPS=2"; do
    env $cfg timeout -k 10 200 python bench.py --in-flight 1 --no-cpu-baseline --no-compare --steps 200 > gpurun_out/r5p.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc [$cfg]"; tail -5 gpurun_out/r5p.log; exit $rc; }
    echo "[if1 $cfg] $(tail -1 gpurun_out/r5p.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["median_ms_per_step"])')"
  done
done | tee gpurun_out/r5p_groups_if1.txt
