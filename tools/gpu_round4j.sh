#!/bin/bash
# Round-4 (j): does handle churn through the library alone reach the fault (stream pool off)? 90 handles, each eager +
# captured + replayed, without heads; if that passes, with heads. A segfault ends the call (its iteration is in the log).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for h in 0 1; do
  timeout -k 10 500 env DDMI_STREAM_POOL=0 python -u tools/repro/handle_churn.py 90 $h 1 > gpurun_out/hchurn_h$h.log 2>&1
  rc=$?; echo "[hchurn heads=$h] rc=$rc"; tail -2 gpurun_out/hchurn_h$h.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
