#!/bin/bash
# BERT: bench line + kernel profile (compression category after the count-pass rework)
set -u
D=gpurun_out/bert
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --model bert --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --model bert --steps 5 --warmup 3 --no-bf16-phase > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker reduce_records_kernel --steps 5 $(find $D/prof -name '*.db' | head -1) $D/kernel_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
find $D/prof -name '*.db' -delete
head -16 $D/kernel_summary.txt
