#!/bin/bash
# ResNet-50 bs32 fp32 (the reference's exp_configs batch): kernel profile
set -u
D=gpurun_out/bs32
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --batch-size 32 --steps 10 --warmup 5 --no-bf16-phase > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker reduce_records_kernel --steps 10 $(find $D/prof -name '*.db' | head -1) $D/prof_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
find $D/prof -name '*.db' -delete
head -14 $D/prof_summary.txt
