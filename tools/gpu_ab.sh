#!/bin/bash
# Same-box bench A/B of environment switches (read at graph capture), alternating REPS times:
#   TAG=r5aa REPS=2 bash tools/gpu_ab.sh "X=0" "DDMI_X5_DEEP=1"
# prints, per run, the 3-lane value, conv_x5 / conv_x6 device ms per step and the in-flight-1 value
# (IF1=0 skips the in-flight-1 leg). PRE: an optional command run first (e.g. a micro A/B under rocprofv3).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=${TAG:-ab}
if [ -n "${PRE:-}" ]; then
  timeout -k 10 400 bash -c "$PRE" > gpurun_out/${T}_pre.log 2>&1
  rc=$?; echo "[pre] rc=$rc"; tail -12 gpurun_out/${T}_pre.log; [ $rc -ne 0 ] && exit $rc
fi
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --steps 100 > gpurun_out/${T}.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc [$cfg]"; tail -5 gpurun_out/${T}.log; exit $rc; }
    echo "[if3 $cfg] $(tail -1 gpurun_out/${T}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); m=d["device_ms_per_step"]; print(d["value"], "x5", m.get("conv_x5"), "x6", m.get("conv_x6"), "x3", m.get("conv_x3"), "tail", m.get("gpt_tail"), "frac", d["roofline"]["frac"])')"
    if [ "${IF1:-1}" != "0" ]; then
      env $cfg timeout -k 10 300 python bench.py --in-flight 1 --no-cpu-baseline --no-compare --steps 200 > gpurun_out/${T}1.log 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc [$cfg]"; tail -5 gpurun_out/${T}1.log; exit $rc; }
      echo "[if1 $cfg] $(tail -1 gpurun_out/${T}1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
    fi
  done
done | tee gpurun_out/${T}_ab.txt
