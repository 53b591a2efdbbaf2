# round 6 (ah): union value_proj phase stamps (DDMI_BUILD_VARIANT=vust), previous build vs residue-class slots
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for v in old new; do
  if [ $v = old ]; then L="$R/tools/micro/ab/old/libddmi_vust.so"; else L="$R/tools/micro/ab/new/libddmi_vust.so"; fi
  echo "[$v]"
  DDMI_LIB=$L timeout -k 10 300 python tools/micro/vu_stamps.py > gpurun_out/r6ah_$v.log 2>&1 || { tail -20 gpurun_out/r6ah_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r6ah_$v.log
done
