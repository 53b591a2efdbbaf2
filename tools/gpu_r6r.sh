# round 6 (r): conv_x6 A/B against the previous build (tools/micro/ab/old/libddmi.so): conv_bench 3x3 shapes, alternating, then the bench
# error vs the fp32 kernel) against the previous build (tools/micro/ab/old/libddmi.so), alternating, then the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for v in old new old new; do
  if [ $v = old ]; then L="$R/tools/micro/ab/old"; else L="$R/diffusiondrive_amd"; fi
  LD_LIBRARY_PATH=$L timeout -k 10 120 ./tools/micro/conv_bench 20 3x3 > gpurun_out/r6r_$v.log 2>&1 || { cat gpurun_out/r6r_$v.log; exit 1; }
  echo "[$v]"; grep -v amdgpu.ids gpurun_out/r6r_$v.log
done
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r6r_bench.json 2> gpurun_out/r6r_bench.err || { tail -5 gpurun_out/r6r_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r6r_bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], 'if1', d['in_flight_1']['value'], 'b1', d.get('batch1_ms'), 'x6 frac', d['roofline']['frac'], d['roofline']['avg_launch_ms'], 'flags', d.get('numerics_flags'), 'l2', d.get('waypoint_l2_vs_oracle'))
print(json.dumps(d['device_ms_per_step']))"
