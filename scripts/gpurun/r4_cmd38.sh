#!/bin/bash
# r4 call 38: bf16 BN-backward GEMM epilogue prefetch -- bf16 GEMM / BN-link tests, interleaved bf16 A/B vs HEAD
set -u
D=gpurun_out/r4c38
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bnlink_gpu.py tests/test_gemm_f32_gpu.py tests/test_kernels2_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -1 $D/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=$D/ab AB_CUT=120 AB_CMDS="python3 bench.py --amp bf16 --steps 20 --warmup 5 --no-bf16-phase --ref-batch 0" bash scripts/gpurun/ab.sh
