#!/bin/bash
# One GPU-box session: op + parity tests, bench, rocprof kernel trace. Stops at the first abnormal exit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$name] abnormal exit ($rc): stopping"; exit $rc; fi
  return $rc
}
step tests 900 python -u -m pytest tests -v -m gpu -x -rf --timeout 300 --timeout-method thread || exit 1
step bench 600 python bench.py ${BENCH_ARGS:-}
cd /tmp && export TMPDIR=/tmp
# single-stream replays (DDMI_STREAMS=0) so per-kernel durations match bench.py's profiled replay; no fp32 leg
DDMI_STREAMS=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof" -o run -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-compare --in-flight 1 > "$R/gpurun_out/prof.log" 2>&1
rc=$?; echo "[rocprof] rc=$rc"; tail -2 "$R/gpurun_out/prof.log"; exit $rc
