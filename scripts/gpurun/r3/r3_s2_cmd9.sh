#!/bin/bash
# batched fp32 BN-backward epilogue loads: GEMM tests, fp32 bench with tune dump (fresh autotune)
set -u
D=gpurun_out/s2k
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f32_gpu.py tests/test_bnlink_gpu.py tests/test_conv1x1_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 $D/tests.log
[ $rc -eq 0 ] || exit $rc
export GKSGD_GEMM_SAVE=$D/choices.json GKSGD_GEMM_DUMP=$D/tune_dump.json GKSGD_GEMM_RETUNE=1
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-400
