#!/bin/bash
# r4 call 2: fp32 32x64-tile family tests, bench (ref_bs32 with the new tiles), bf16-phase isolation, bs32 profile
set -u
D=gpurun_out/r4c2
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gemm_f32_gpu.py tests/test_bench_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
GKSGD_GEMM_SAVE=$D/gemm_choices.json GKSGD_GEMM_DUMP=$D/gemm_dump.json timeout -k 10 400 python3 bench.py --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; cat $D/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --ref-batch 0 --json-out $D/bench_noref.json > $D/bench_noref.log 2>&1
rc=$?; echo bench2_rc=$rc; python3 -c "import json;d=json.load(open('$D/bench_noref.json'));print('noref', d['value'], d.get('bf16_value'), d.get('bf16_ms_per_step'))"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --batch-size 32 --steps 10 --warmup 5 --no-bf16-phase --ref-batch 0 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker reduce_records_kernel --steps 10 --sequence $D/seq_bs32.csv $(find $D/prof -name '*.db' | head -1) $D/prof_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
find $D/prof -name '*.db' -delete
head -12 $D/prof_summary.txt
