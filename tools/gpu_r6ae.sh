# round 6 (ae): conv_x6 BAR2 (barriers at even taps, 5-slot ring) on the 8 x 8 LiDAR layer-4 form: conv op tests,
# conv_bench A/B against the previous build (tools/micro/ab/old/libddmi.so), then the bench, old / new alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "conv" > gpurun_out/r6ae_tests.log 2>&1 || { tail -30 gpurun_out/r6ae_tests.log; exit 1; }
tail -2 gpurun_out/r6ae_tests.log
for v in old new old new; do
  if [ $v = old ]; then L="$R/tools/micro/ab/old"; else L="$R/diffusiondrive_amd"; fi
  LD_LIBRARY_PATH=$L timeout -k 10 120 ./tools/micro/conv_bench 40 lid.l4 > gpurun_out/r6ae_$v.log 2>&1 || { cat gpurun_out/r6ae_$v.log; exit 1; }
  echo "[$v]"; grep -v amdgpu.ids gpurun_out/r6ae_$v.log
done
for v in old new old new; do
  if [ $v = old ]; then L="$R/tools/micro/ab/old/libddmi.so"; else L="$R/diffusiondrive_amd/libddmi.so"; fi
  DDMI_LIB=$L timeout -k 10 400 python bench.py --no-cpu-baseline --no-compare > gpurun_out/r6ae_b$v.json 2> gpurun_out/r6ae_b$v.err || { tail -5 gpurun_out/r6ae_b$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r6ae_b$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], 'ms', d['ms_per_step'], 'x6', d['roofline']['frac'], d['roofline']['avg_launch_ms'], 'flags', d.get('numerics_flags'))" || exit 1
done
