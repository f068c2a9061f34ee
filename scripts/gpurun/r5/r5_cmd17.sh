#!/bin/bash
# r5c17: compression pipeline kernel trace on the 25.6 M bucket (default hand-off)
set -u
D=gpurun_out/r5c17
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/p -o p -- python3 scripts/debug/compress_prof.py > $D/p.log 2>&1
rc=$?; echo rc=$rc; [ $rc -eq 0 ] || { tail $D/p.log; exit $rc; }
python3 scripts/debug/compress_prof.py --summarize $D/p > $D/sum.txt 2>&1; cat $D/sum.txt
