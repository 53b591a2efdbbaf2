# round 6 (b): the memset-node failure of tfdec_mk4 replays, traced: rocprofv3 kernel trace of tf_replay with the
# memset node (is the fill dispatch done before tfdec_mk4 starts?), and the same run with the runtime's graph packet
# capture off
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
DDMI_TF_MEMSET=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6b_trace -o run -- python3 -u tools/debug/tf_replay.py > gpurun_out/r6b_tfr_trace.log 2>&1 && \
DDMI_TF_MEMSET=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 python -u tools/debug/tf_replay.py > gpurun_out/r6b_tfr_nopc.log 2>&1
rc=$?; grep -c "same-as-first False\|flags [1-9]" gpurun_out/r6b_tfr_trace.log; grep -c "flags [1-9]" gpurun_out/r6b_tfr_nopc.log; grep "streams 2" gpurun_out/r6b_tfr_nopc.log | head -12; find gpurun_out/r6b_trace -name "*.csv" | head; exit $rc
