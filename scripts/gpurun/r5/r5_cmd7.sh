#!/bin/bash
# r5c7: compression pipeline (25.6 M bucket, gaussian, launch and in-grid hand-offs) kernel trace
set -u
D=gpurun_out/r5c7
mkdir -p $D
export TMPDIR=/tmp
for H in launch lastblock; do
  GKSGD_HANDOFF=$H timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/p_$H -o p -- python3 scripts/debug/compress_prof.py > $D/p_$H.log 2>&1
  rc=$?; echo ${H}_rc=$rc; [ $rc -eq 0 ] || exit $rc
  python3 scripts/debug/compress_prof.py --summarize $D/p_$H > $D/sum_$H.txt 2>&1; cat $D/sum_$H.txt
done
