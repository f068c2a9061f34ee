#!/bin/bash
# r5c18: BERT-base fp32 (bucketed compression): native vs bf16x6 GEMM candidates; x6 kernel profile
set -u
D=gpurun_out/r5c18
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --model bert --steps 10 --warmup 3 --no-bf16-phase"
timeout -k 10 400 $B --f32-matmul native --json-out $D/native.json > $D/native.log 2>&1
rc=$?; echo native_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/native.log; exit $rc; }
GKSGD_GEMM_SAVE=$D/choices.json GKSGD_GEMM_DUMP=$D/dump.json timeout -k 10 500 $B --f32-matmul bf16x6 --json-out $D/x6.json > $D/x6.log 2>&1
rc=$?; echo x6_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/x6.log; exit $rc; }
python3 -c "
import json
for n in ('native','x6'):
    d=json.load(open('$D/%s.json'%n)); print(n, d['value'], d['ms_per_step'])"
GKSGD_GEMM_CACHE=$D/choices.json timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- $B --steps 10 --f32-matmul bf16x6 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker reduce_records_kernel --steps 10 $(find $D/prof -name '*.db' | head -1) $D/prof_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
head -30 $D/prof_summary.txt | cut -c1-220
