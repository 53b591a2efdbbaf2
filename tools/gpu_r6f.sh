# round 6 (f): the memset-node reproducer at the product's counter sizes (B = 8: 16 words; B = 1: 2 words), then the
# bench with the batch-1 leg
set -o pipefail
for w in 16 2 64; do
  timeout -k 10 120 ./tools/repro/memset_node 500 20 - $w > gpurun_out/r6f_memset_w$w.log 2>&1 || exit $?
  echo "words $w:"; grep "case [78]" gpurun_out/r6f_memset_w$w.log
done
timeout -k 10 600 python -u bench.py > gpurun_out/r6f_bench.json 2> gpurun_out/r6f_bench.err
rc=$?; tail -c 400 gpurun_out/r6f_bench.err; python -c "
import json; d=json.loads(open('gpurun_out/r6f_bench.json').read().strip().splitlines()[-1]); print('value', d['value'], 'if1', d.get('in_flight_1',{}).get('value'), 'batch1', d.get('batch1')); print('roofline', d['roofline']['achieved'], d['roofline']['frac'])"; exit $rc
