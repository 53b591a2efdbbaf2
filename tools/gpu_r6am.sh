# round 6 (am): union value_proj on 4 waves of 64 x 128 (one wave per SIMD, accumulators in AGPRs) built as
# tools/micro/ab/new/libddmi.so, against the in-tree build: value_proj / golden tests on the new build, whole-forward
# bit identity, kernel trace of the forward, bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/r6am
OLD=$R/diffusiondrive_amd/libddmi.so; NEW=$R/tools/micro/ab/new/libddmi.so
DDMI_LIB=$NEW timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -v -m gpu --timeout 240 --timeout-method thread -k "value or goldens or batch8 or replays" > gpurun_out/r6am/tests.log 2>&1 || { tail -40 gpurun_out/r6am/tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6am/tests.log | tail -2
DDMI_LIB=$OLD OUT=gpurun_out/r6am/old.json timeout -k 10 300 python tools/micro/model_ab.py > gpurun_out/r6am/mold.log 2>&1 || { tail -20 gpurun_out/r6am/mold.log; exit 1; }
DDMI_LIB=$NEW OUT=gpurun_out/r6am/new.json REF=gpurun_out/r6am/old.json timeout -k 10 300 python tools/micro/model_ab.py > gpurun_out/r6am/mnew.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6am/mnew.log; [ $rc = 0 ] || exit 1
for v in old new; do
  if [ $v = old ]; then L=$OLD; else L=$NEW; fi
  (cd /tmp && export TMPDIR=/tmp && DDMI_LIB=$L OUT=/tmp/ab_$v.json timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/r6am/t_$v" -o run -- python "$R/tools/micro/model_ab.py" > "$R/gpurun_out/r6am/t_$v.log" 2>&1) || { tail -5 gpurun_out/r6am/t_$v.log; exit 1; }
  echo "[trace $v]"; python tools/kstats.py gpurun_out/r6am/t_$v --grep vproj
done
for v in old new old new; do
  if [ $v = old ]; then L=$OLD; else L=$NEW; fi
  DDMI_LIB=$L timeout -k 10 400 python bench.py --no-cpu-baseline --no-compare > gpurun_out/r6am/b$v.json 2> gpurun_out/r6am/b$v.err || { tail -5 gpurun_out/r6am/b$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r6am/b$v.json').read().strip().splitlines()[-1])
v=d['decoder_cross_attention']
print('$v', d['value'], 'ms', d['ms_per_step'], 'vproj', v['avg_launch_ms'], v['live_mfma_equiv_util'], 'flags', d.get('numerics_flags'))" || exit 1
done
