#!/bin/bash
set -u
D=gpurun_out/r3k
mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1_gpu.py tests/test_bn_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log
[ $rc -eq 0 ] || exit $rc
export GKSGD_GEMM_SAVE=$D/choices.json GKSGD_GEMM_DUMP=$D/tune_dump.json
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-400
