#!/bin/bash
# Winograd fp32 kernel tests, GPU suite, fp32 bench (choices saved), fp32 profile
set -u
D=gpurun_out/s2b
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_winograd_gpu.py > $D/wino_tests.log 2>&1
rc=$?; echo wino_tests_rc=$rc; tail -3 $D/wino_tests.log
[ $rc -eq 0 ] || exit $rc
export GKSGD_GEMM_SAVE=$D/choices.json GKSGD_GEMM_DUMP=$D/tune_dump.json
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
unset GKSGD_GEMM_SAVE GKSGD_GEMM_DUMP
export GKSGD_GEMM_CACHE=$PWD/$D/choices.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D/prof_fp32 -o run -- python3 bench.py --steps 10 --warmup 3 --no-bf16-phase > $D/prof_fp32.log 2>&1
echo prof_rc=$?
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log
