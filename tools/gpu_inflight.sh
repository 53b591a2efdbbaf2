set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_inflight_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_if.log 2>&1; rc=$?; tail -3 gpurun_out/t_if.log; [ $rc -ne 0 ] && exit $rc
for n in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --in-flight $n > gpurun_out/b_if$n.json 2> gpurun_out/b_if$n.err || { tail -5 gpurun_out/b_if$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/b_if$n.json').read().strip().splitlines()[-1]);print($n, d['value'], d['ms_per_step'], d['median_ms_per_step'], d['median_batch_latency_ms'], d['roofline']['frac'])"
done
