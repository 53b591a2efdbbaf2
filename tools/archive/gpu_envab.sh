#!/bin/bash
# Same-box A/B of runtime knobs through the bench: gpu_envab.sh "ENV=a ENV2=b" "ENV=c" ...  (each argument is one
# configuration's environment; the first runs again at the end). Prints value, ms/step, the in_flight_1 value (NOCMP=
# runs the compare legs) and device ms per class.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
i=0
for cfg in "$@" "$1"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python bench.py --steps ${STEPS:-100} --no-cpu-baseline ${NOCMP---no-compare} ${BENCH_EXTRA:-} > gpurun_out/envab_$i.log 2>&1 || { tail -5 gpurun_out/envab_$i.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/envab_$i.log').read().strip().splitlines()[-1]);dm=d['device_ms_per_step'];print('[$cfg]', d['value'], d['ms_per_step'], (d.get('in_flight_1') or {}).get('value'), {k: round(v,3) for k,v in dm.items()})"
done
