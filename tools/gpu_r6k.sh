# round 6 (k): the one-channel LiDAR stem with split accumulators as the default - parity (the whole parity file, the
# stem op tests), the diagnosis script, then the bench with it and without it (DDMI_STEM1=0)
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py "tests/test_ops_gpu.py::test_stem_pool_nchw" > gpurun_out/r6k_tests.log 2>&1 || { tail -30 gpurun_out/r6k_tests.log; exit 1; }
tail -3 gpurun_out/r6k_tests.log
timeout -k 10 300 python -u tools/debug/stem1_diag.py > gpurun_out/r6k_stem1.log 2>&1 && cat gpurun_out/r6k_stem1.log || exit 1
for v in 1 0 1; do
  DDMI_STEM1=$v timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r6k_bench_stem$v.json 2> gpurun_out/r6k_bench_stem$v.err || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/r6k_bench_stem$v.json').read().strip().splitlines()[-1])
print('STEM1=$v', d['value'], d['in_flight_1']['value'], d['batch1']['median_ms'], d['device_ms_per_step'].get('stem_pool'))"
done
