# round 6 (al): GPT attention with an XCD-aware workgroup order (the two workgroups of a (scene, head) at head size 128
# on one XCD): whole-forward bit identity against the previous build, kernel trace of the attention, bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/r6al
OLD=$R/tools/micro/ab/old/libddmi.so
DDMI_LIB=$OLD OUT=gpurun_out/r6al/old.json timeout -k 10 300 python tools/micro/model_ab.py > gpurun_out/r6al/mold.log 2>&1 || { tail -20 gpurun_out/r6al/mold.log; exit 1; }
OUT=gpurun_out/r6al/new.json REF=gpurun_out/r6al/old.json timeout -k 10 300 python tools/micro/model_ab.py > gpurun_out/r6al/mnew.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6al/mnew.log; [ $rc = 0 ] || exit 1
for v in old new; do
  if [ $v = old ]; then L=$OLD; else L="$R/diffusiondrive_amd/libddmi.so"; fi
  (cd /tmp && export TMPDIR=/tmp && DDMI_LIB=$L OUT=/tmp/ab_$v.json timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/r6al/t_$v" -o run -- python "$R/tools/micro/model_ab.py" > "$R/gpurun_out/r6al/t_$v.log" 2>&1) || { tail -5 gpurun_out/r6al/t_$v.log; exit 1; }
  echo "[trace $v]"; python tools/kstats.py gpurun_out/r6al/t_$v --grep gpt_attn
done
for v in old new old new; do
  if [ $v = old ]; then L=$OLD; else L="$R/diffusiondrive_amd/libddmi.so"; fi
  DDMI_LIB=$L timeout -k 10 400 python bench.py --no-cpu-baseline --no-compare > gpurun_out/r6al/b$v.json 2> gpurun_out/r6al/b$v.err || { tail -5 gpurun_out/r6al/b$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r6al/b$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], 'ms', d['ms_per_step'], 'flags', d.get('numerics_flags'))" || exit 1
done
