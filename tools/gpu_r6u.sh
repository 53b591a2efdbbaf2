# round 6 (u): the stride-2 direct conv (conv_x6 phase halos) - conv_bench s2 shapes against the previous build
# (implicit GEMM), the conv op tests and the parity goldens, then the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for v in old new old new; do
  if [ $v = old ]; then L="$R/tools/micro/ab/old"; else L="$R/diffusiondrive_amd"; fi
  LD_LIBRARY_PATH=$L timeout -k 10 120 ./tools/micro/conv_bench 20 s2 > gpurun_out/r6u_$v.log 2>&1 || { cat gpurun_out/r6u_$v.log; exit 1; }
  echo "[$v]"; grep -v amdgpu.ids gpurun_out/r6u_$v.log
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_parity_gpu.py > gpurun_out/r6u_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r6u_tests.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAIL" gpurun_out/r6u_tests.log | head -80; exit $rc; }
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r6u_bench.json 2> gpurun_out/r6u_bench.err || { tail -5 gpurun_out/r6u_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r6u_bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], 'if1', d['in_flight_1']['value'], 'b1', d.get('batch1_ms'), 'x6 frac', d['roofline']['frac'], d['roofline']['avg_launch_ms'], 'flags', d.get('numerics_flags'))
print(json.dumps(d['device_ms_per_step']))"
