#!/bin/bash
# Same-box A/B of the launch-stream priority in two-stream mode: batch-1 latency (tools/bench_configs.py child mode)
# and one B = 64 batch at a time (bench.py --in-flight 1), a fresh process each. Arguments: DDMI_MAIN_PRIORITY values
# ("" = the default, greatest).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for p in "$@"; do
  out=$(env DDMI_MAIN_PRIORITY=$p timeout -k 10 200 python tools/bench_configs.py --c1-two-stream --steps 20 2>&1 | grep '^C1TWO') || { echo "[prio=$p] C1 failed"; exit 1; }
  echo "[prio=$p] $out"
  env DDMI_MAIN_PRIORITY=$p timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-compare --in-flight 1 > gpurun_out/abc1_$p.log 2>&1 || { tail -5 gpurun_out/abc1_$p.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/abc1_$p.log').read().strip().splitlines()[-1]);print('[prio=$p] B64 in-flight 1:', d['value'], d['ms_per_step'])"
done
