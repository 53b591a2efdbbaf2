# round 6 (c): which part of the memset node breaks tfdec_mk4 replays (DDMI_TF_MEMSET modes, tfdec_mk.hip)
set -o pipefail
for m in 1 2 3 4; do
  DDMI_TF_MEMSET=$m timeout -k 10 240 python -u tools/debug/tf_replay.py > gpurun_out/r6c_tfr_m$m.log 2>&1 || exit $?
  echo "mode $m: $(grep -c 'same-as-first False\|flags [1-9]' gpurun_out/r6c_tfr_m$m.log) bad lines of 36; flags: $(grep -o 'flags [0-9]*' gpurun_out/r6c_tfr_m$m.log | sort | uniq -c | tr '\n' ' ')"
done
