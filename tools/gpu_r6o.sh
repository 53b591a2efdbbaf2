# round 6 (o): the stem with its fragment reads two units ahead - bit-identity against the previous build
# (tools/micro/ab/old/libddmi.so), stem op tests, then both builds' stem kernels under the kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
OLD=$R/tools/micro/ab/old/libddmi.so
DDMI_LIB=$OLD OUT=gpurun_out/r6o_old.json timeout -k 10 200 python tools/micro/stem_ab.py > gpurun_out/r6o_ab.log 2>&1 || { cat gpurun_out/r6o_ab.log; exit 1; }
OUT=gpurun_out/r6o_new.json REF=gpurun_out/r6o_old.json timeout -k 10 200 python tools/micro/stem_ab.py >> gpurun_out/r6o_ab.log 2>&1 || { cat gpurun_out/r6o_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6o_ab.log
true
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  if [ $v = old ]; then export DDMI_LIB=$OLD; else unset DDMI_LIB; fi
  OUT=/tmp/x.json timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r6o_$v" -- python3 "$R/tools/micro/stem_ab.py" > "$R/gpurun_out/r6o_$v.log" 2>&1 || exit 1
  echo "[$v]"; python3 "$R/tools/kstats.py" "$R/gpurun_out/r6o_$v" --grep stem_pool
done
