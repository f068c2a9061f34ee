#!/bin/bash
# tests after non-temporal BN + autotune margin; fp32 headline bench (choices
# saved), profile of the fp32 step with those choices, PMC counters
set -u
D=gpurun_out/r3n
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bn_gpu.py tests/test_bnlink_gpu.py \
  tests/test_conv1x1_gpu.py tests/test_gemm_f32_gpu.py tests/test_stem_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 $D/tests.log
[ $rc -eq 0 ] || exit $rc
export GKSGD_GEMM_SAVE=$D/choices.json GKSGD_GEMM_DUMP=$D/tune_dump.json
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
unset GKSGD_GEMM_SAVE GKSGD_GEMM_DUMP
export GKSGD_GEMM_CACHE=$PWD/$D/choices.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof_fp32 -o run -- python3 bench.py --steps 10 --warmup 3 --no-bf16-phase > $D/prof_fp32.log 2>&1
echo prof_rc=$?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof_bf16 -o run -- python3 bench.py --amp bf16 --steps 10 --warmup 3 --no-bf16-phase > $D/prof_bf16.log 2>&1
echo prof16_rc=$?
