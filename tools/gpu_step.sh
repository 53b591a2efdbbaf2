#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first failure.
#   gpu_step.sh "name:timeout:command" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; to=${rest%%:*}; cmd=${rest#*:}
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[$name] rc=$rc"; tail -${TAILN:-6} "gpurun_out/$name.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
