#!/bin/bash
# r4 call 35: bf16 ResNet-50 bs512 kernel profile on the final round-4 build
set -u
D=gpurun_out/r4c35
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --amp bf16 --steps 10 --warmup 5 --no-bf16-phase --ref-batch 0 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker reduce_records_kernel --steps 10 $(find $D/prof -name '*.db' | head -1) $D/prof_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
head -12 $D/prof_summary.txt
tail -1 $D/prof.log | cut -c1-200
