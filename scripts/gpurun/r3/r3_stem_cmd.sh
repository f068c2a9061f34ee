#!/bin/bash
# fp32 stem kernels: numerics tests, fp32 headline bench, kernel profile
set -u
D=gpurun_out/stem
mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_stem_gpu.py > $D/tests.log 2>&1
rc=$?; echo stem_tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-bf16-phase --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
GKSGD_STEM_F32=0 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-bf16-phase --json-out $D/bench_nof32.json > $D/bench_nof32.log 2>&1
rc=$?; echo bench_nof32_rc=$rc; tail -1 $D/bench_nof32.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --steps 5 --warmup 3 --no-bf16-phase > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker reduce_records_kernel --steps 5 $(find $D/prof -name '*.db' | head -1) $D/prof_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
find $D/prof -name '*.db' -delete
grep -i "stem\|miopen\|Naive\|igemm" $D/prof_summary.txt > $D/stem_rows.txt; cat $D/stem_rows.txt
echo done
