#!/bin/bash
# round 5q: fused BasicBlock per trunk (DDMI_BB_FUSE 0 / 2 = LiDAR / 3 = camera), same box, alternating
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "DDMI_BB_FUSE=0" "DDMI_BB_FUSE=2" "DDMI_BB_FUSE=3"; do
    env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --steps 100 > gpurun_out/r5q.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc [$cfg]"; tail -5 gpurun_out/r5q.log; exit $rc; }
    echo "[if3 $cfg] $(tail -1 gpurun_out/r5q.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); dm=d["device_ms_per_step"]; print(d["value"], d["in_flight_1"]["value"] if d.get("in_flight_1") else None, dm["conv_x6"], dm.get("basicblock"))')"
  done
done | tee gpurun_out/r5q_bbfuse.txt
