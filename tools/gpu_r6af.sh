# round 6 (af, ai): union value_proj A/B (af: residue-class union slots; ai: cross-term MFMAs ahead of the step barrier):
# golden tests, whole-forward bit identity against the previous build (tools/micro/ab/old/libddmi.so), bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -v -m gpu --timeout 240 --timeout-method thread -k "value or goldens or batch8 or replays" > gpurun_out/r6af_tests.log 2>&1 || { tail -40 gpurun_out/r6af_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6af_tests.log | tail -3
DDMI_LIB=$R/tools/micro/ab/old/libddmi.so OUT=gpurun_out/r6af_old.json timeout -k 10 300 python tools/micro/model_ab.py > gpurun_out/r6af_mold.log 2>&1 || { tail -20 gpurun_out/r6af_mold.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6af_mold.log
OUT=gpurun_out/r6af_new.json REF=gpurun_out/r6af_old.json timeout -k 10 300 python tools/micro/model_ab.py > gpurun_out/r6af_mnew.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6af_mnew.log
[ $rc = 0 ] || exit 1
for v in old new old new; do
  if [ $v = old ]; then L="$R/tools/micro/ab/old/libddmi.so"; else L="$R/diffusiondrive_amd/libddmi.so"; fi
  DDMI_LIB=$L timeout -k 10 400 python bench.py --no-cpu-baseline --no-compare > gpurun_out/r6af_b$v.json 2> gpurun_out/r6af_b$v.err || { tail -5 gpurun_out/r6af_b$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r6af_b$v.json').read().strip().splitlines()[-1])
v=d['decoder_cross_attention']
print('$v', d['value'], 'ms', d['ms_per_step'], 'vproj', v['avg_launch_ms'], v['live_mfma_equiv_util'], 'flags', d.get('numerics_flags'))" || exit 1
done
