#!/bin/bash
# conv_x6 activation cache policy (DDMI_X6_NT, read per dispatch) on the conv micro-benchmark, per trunk shape,
# then FETCH_SIZE of the main image shapes under each policy (one rocprofv3 --pmc pass each).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/x6nt.log; : > $out
for shp in ${SHAPES:-img.l1.3x3 img.l2.3x3 img.l3.3x3 img.l4.3x3 lid.l1.3x3 lid.l3.3x3}; do
  for v in 0 1 2 3 0; do
    r=$(DDMI_X6_NT=$v timeout -k 5 60 tools/micro/conv_bench ${REPS:-30} $shp 2>&1 | tail -1)
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $shp $v"; exit $rc; }
    echo "nt=$v $r" | tee -a $out
  done
done
