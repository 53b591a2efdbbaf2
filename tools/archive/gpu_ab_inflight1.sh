set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
run() { local tag=$1; shift; env "$@" > /dev/null; timeout -k 10 200 env "${ENVS[@]}" python bench.py --steps 100 --no-cpu-baseline $EXTRA > gpurun_out/ab7_$tag.log 2>&1 || { tail -5 gpurun_out/ab7_$tag.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab7_$tag.log').read().strip().splitlines()[-1]);print('[$tag]', d['value'], d['ms_per_step'], (d.get('in_flight_1') or {}).get('value'))"; }
ENVS=(DDMI_NONE=0); EXTRA="--in-flight 1 --no-compare"; run if1_lazy
ENVS=(DDMI_MAIN_PRIORITY=0); EXTRA="--in-flight 1 --no-compare"; run if1_prio0
ENVS=(DDMI_STREAMS=0); EXTRA="--in-flight 1 --no-compare"; run if1_single
ENVS=(DDMI_NONE=0); EXTRA="--in-flight 1 --no-compare"; run if1_lazy_again
