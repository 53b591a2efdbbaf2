# round 6 (ad): lanes with two-stream captured forwards (--lane-streams 2) against single-stream lanes, 3 in flight
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for ls in 1 2 1 2; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --no-compare --lane-streams $ls > gpurun_out/r6ad_$ls.json 2> gpurun_out/r6ad_$ls.err || { tail -5 gpurun_out/r6ad_$ls.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r6ad_$ls.json').read().strip().splitlines()[-1])
print('lane_streams=$ls', d['value'], 'ms', d['ms_per_step'], 'median batch latency', d.get('median_batch_latency_ms'))" || exit 1
done
