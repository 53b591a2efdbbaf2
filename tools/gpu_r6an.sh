# round 6 (an): decoder_mk with two query-group workgroups per scene at B = 64 (DDMI_MK_GROUPS=2; default 1 there)
# against the default: bench alternating (3 in flight and one at a time), decoder device time, oracle L2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/r6an
for g in 1 2 1 2; do
  DDMI_MK_GROUPS=$g timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r6an/b$g.json 2> gpurun_out/r6an/b$g.err || { tail -5 gpurun_out/r6an/b$g.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r6an/b$g.json').read().strip().splitlines()[-1])
print('groups=$g', d['value'], 'if1', d.get('in_flight_1', {}).get('value'), 'decoder ms', d['device_ms_per_step']['decoder'], 'L2', d.get('waypoint_l2_vs_oracle'), 'flags', d.get('numerics_flags'))" || exit 1
done
