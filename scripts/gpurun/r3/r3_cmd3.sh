#!/bin/bash
set -u
mkdir -p gpurun_out/r3c
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bnlink_gpu.py \
  tests/test_kernels_gpu.py tests/test_e2e_gpu.py tests/test_conv1x1_gpu.py tests/test_stem_gpu.py \
  tests/test_bn_gpu.py > gpurun_out/r3c/tests2.log 2>&1
rc=$?; echo tests_rc=$rc; tail -5 gpurun_out/r3c/tests2.log
exit $rc
