#!/bin/bash
# GPU box: gpu tests, then bench once per env setting given as arguments ("" = default). Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
if [ -z "${NOTESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -rf --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
fi
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare ${BENCH_ARGS:-} > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err
  rc=$?; echo "[$e] rc=$rc"; python -c "
import json,sys; r=json.load(open('gpurun_out/ab_$i.json')); print(r['value'], r['ms_per_step'], r['roofline']['frac'], r.get('device_ms_per_step'))"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
