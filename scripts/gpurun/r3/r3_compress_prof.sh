#!/bin/bash
# compression pipeline: per-kernel rocprofv3 breakdown of bench/kernels.py round2
set -u
D=gpurun_out/cprof
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench/kernels.py --only ${ONLY:-round2} > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --steps 1 --top 40 $(find $D/prof -name '*.db' | head -1) $D/kernel_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
find $D/prof -name '*.db' -delete
cut -c1-200 $D/kernel_summary.txt | head -50
