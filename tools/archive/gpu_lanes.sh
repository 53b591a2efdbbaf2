#!/bin/bash
# Lanes sweep on the final tree (same box): bench --in-flight 2 / 3 / 4 / 3, 100 steps each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for n in 2 3 4 3; do
  timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --no-compare --in-flight $n > gpurun_out/lanes_$n.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/lanes_$n.log').read().strip().splitlines()[-1]);print('in_flight $n', d['value'], d['ms_per_step'], d['median_batch_latency_ms'])" | tee -a gpurun_out/lanes.txt
done
