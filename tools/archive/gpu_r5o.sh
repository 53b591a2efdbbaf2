#!/bin/bash
# round 5o: lanes A/B with the segmented programs - lanes x streams per lane (same box, alternating)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "--in-flight 3" "--in-flight 3 --lane-streams 2" "--in-flight 2 --lane-streams 2" "--in-flight 4"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --steps 100 $cfg > gpurun_out/r5o.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc [$cfg]"; tail -5 gpurun_out/r5o.log; exit $rc; }
    echo "[$cfg] $(tail -1 gpurun_out/r5o.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["median_batch_latency_ms"])')"
  done
done | tee gpurun_out/r5o_lanes.txt
