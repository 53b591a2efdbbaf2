#!/bin/bash
# Round-3 (m) evidence: tools/gpu_all.sh (GPU tests, bench, rocprof trace), then the C2-bf16 / C4 configs with
# batches in flight. Stops at the first abnormal exit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
bash tools/gpu_all.sh || exit $?
cd "$R"
for cfg in "--gemm bf16" "--arch resnet50 --gemm bf16" "--arch resnet50 --gemm f16x3"; do
  for n in 1 3; do
    tag=$(echo "$cfg $n" | tr -d '-' | tr ' ' '_')
    timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --no-compare --in-flight $n $cfg > gpurun_out/cfg_$tag.json 2> gpurun_out/cfg.err || { tail -5 gpurun_out/cfg.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/cfg_$tag.json').read().strip().splitlines()[-1]);print('[$cfg] in_flight $n', d['value'], d['ms_per_step'], d['median_batch_latency_ms'])"
  done
done
