#!/bin/bash
# conv path change: GPU conv tests + fp32 headline bench
set -u
D=gpurun_out/cab2
mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv1x1_gpu.py tests/test_winograd_gpu.py tests/test_gemm_f32_gpu.py tests/test_bn_lazy_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-bf16-phase --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
echo done
