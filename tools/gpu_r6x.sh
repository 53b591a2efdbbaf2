# round 6 (x): same-box bench A/B of the session's start (tools/micro/ab/old/libddmi.so, tree f5862a5) against the
# current build, alternating: 3 in flight and one at a time
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for v in old new old new; do
  if [ $v = old ]; then export DDMI_LIB=$R/tools/micro/ab/old/libddmi.so; else unset DDMI_LIB; fi
  for L in 3 1; do
    timeout -k 10 400 python bench.py --no-cpu-baseline --no-compare --in-flight $L > gpurun_out/r6x_${v}_$L.json 2> gpurun_out/r6x_${v}_$L.err || { tail -5 gpurun_out/r6x_${v}_$L.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r6x_${v}_$L.json').read().strip().splitlines()[-1])
m=d['device_ms_per_step']
print('$v in_flight=$L', d['value'], 'ms', d['ms_per_step'], 'x6', m['conv_x6'], 'x5', m['conv_x5'], 'x3', m['conv_x3'], 'stem', m['stem_pool'])" || exit 1
  done
done
