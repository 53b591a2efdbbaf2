#!/bin/bash
# Batches-in-flight sweep: GPU_MAX_HW_QUEUES x lanes x streams per lane (bench.py, no fp32 / H2D legs).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for q in ${QUEUES:-4 16}; do for n in ${LANES:-3 4}; do for ls in ${LSTREAMS:-1 2}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 150 --no-cpu-baseline --no-compare --in-flight $n --lane-streams $ls > gpurun_out/lanes_${q}_${n}_${ls}.json 2>gpurun_out/lanes.err || { tail -5 gpurun_out/lanes.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/lanes_${q}_${n}_${ls}.json').read().strip().splitlines()[-1]);print('queues $q lanes $n lane_streams $ls', d['value'], d['ms_per_step'], d['median_batch_latency_ms'])"
done; done; done
