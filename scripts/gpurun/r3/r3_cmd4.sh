#!/bin/bash
set -u
mkdir -p gpurun_out/r3d
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bn_lazy_gpu.py \
  > gpurun_out/r3d/lazy.log 2>&1
rc=$?; echo lazy_rc=$rc; tail -30 gpurun_out/r3d/lazy.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_f32_gpu.py \
  tests/test_bnlink_gpu.py tests/test_conv1x1_gpu.py tests/test_bn_gpu.py > gpurun_out/r3d/f32.log 2>&1
rc=$?; echo f32_rc=$rc; tail -5 gpurun_out/r3d/f32.log
exit $rc
