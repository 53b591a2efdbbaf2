#!/bin/bash
# Round-4 (l): the pure-HIP reproducer shaped like the faulting order: a long-lived two-stream handle replayed while
# many handles (two-stream and single-stream on caller streams) are created and destroyed, then the long-lived one
# destroyed and a fresh two-stream handle captured and launched; streams not pooled. Larger graphs, several fork /
# join pairs and memset nodes. A segfault ends the call.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for a in "60 0 64 0 1 0" "60 0 512 0 4 1"; do
  set -- $a
  timeout -k 10 300 tools/repro/graph_churn $a > gpurun_out/churn_long_$2_$3_$5.log 2>&1; rc=$?
  echo "[graph_churn $a] rc=$rc"; tail -2 gpurun_out/churn_long_$2_$3_$5.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 env DDMI_STREAM_POOL=0 python -u tools/repro/handle_churn.py 50 0 1 1 > gpurun_out/hchurn_long.log 2>&1
rc=$?; echo "[hchurn long] rc=$rc"; tail -3 gpurun_out/hchurn_long.log; exit $rc
