# round 6 (w): conv_x5's 128 x 128 two-per-CU routing as the default - op tests, parity goldens, the whole-forward
# bench, and the per-launch table
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_parity_gpu.py > gpurun_out/r6w_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r6w_tests.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAIL" gpurun_out/r6w_tests.log | head -60; exit $rc; }
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r6w_bench.json 2> gpurun_out/r6w_bench.err || { tail -5 gpurun_out/r6w_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r6w_bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], 'if1', d['in_flight_1']['value'], 'b1', d.get('batch1_ms'), 'x6 frac', d['roofline']['frac'], d['roofline']['avg_launch_ms'], 'flags', d.get('numerics_flags'))
print(json.dumps(d['device_ms_per_step']))"
timeout -k 10 300 python tools/launch_log.py --out gpurun_out/r6w_launches.md > gpurun_out/r6w_ll.log 2>&1 && grep "all shapes\|GEMM / conv total" gpurun_out/r6w_launches.md
