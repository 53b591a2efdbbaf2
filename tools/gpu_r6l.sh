# round 6 (l): the union value_proj's K split at B = 64 (DDMI_VPROJ_USPLIT 1 = default there, 2, 4): bench headline,
# one at a time, and the decoder cross-attention record
set -o pipefail
for u in 0 4 2 0 4; do
  if [ $u = 0 ]; then unset DDMI_VPROJ_USPLIT; else export DDMI_VPROJ_USPLIT=$u; fi
  timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r6l_bench_u$u.json 2> gpurun_out/r6l_bench_u$u.err || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/r6l_bench_u$u.json').read().strip().splitlines()[-1]); v=d['decoder_cross_attention']
print('usplit=$u value', d['value'], 'if1', d['in_flight_1']['value'], 'b1', d['batch1']['median_ms'], 'vp avg ms', v['avg_launch_ms'], 'live util', v['live_mfma_equiv_util'], 'flags', d['numerics_flags'])"
done
