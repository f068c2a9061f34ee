#!/bin/bash
# round 3: GPU tests of the new fp32 / overflow / RCCL-failure code, fp32 GEMM
# config sweeps and PMC counters of the fp32 MFMA kernels
set -u
mkdir -p gpurun_out/r3b
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_kernels2_gpu.py tests/test_bench_gpu.py > gpurun_out/r3b/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/r3b/tests.log
[ $rc -eq 0 ] || exit $rc
P="timeout -k 10 120 python bench/gemm_probe.py --dtype f32 --iters 10"
{
$P --op conv --C 64 --H 56 --k 3 --sweep 1,2,3,4,7,11,14,21,24,101,102,104,201,204
$P --op conv --C 256 --H 14 --k 3 --sweep 1,2,3,4,7,11,14,21,24,101,102,104,201,204
$P --op gemm --C 256 --K 64 --H 56 --sweep 1,2,3,4,7,101,102,104,201
$P --op gemm --C 64 --K 256 --H 56 --sweep 1,2,3,4,7,101,102,104,201
$P --op cwgrad --C 64 --H 56 --k 3 --sweep 1,2,3,4,5,6,7,8,9,11,14,16
$P --op cwgrad --C 256 --H 14 --k 3 --sweep 1,2,3,4,5,6,7,8,9,11,14,16
$P --op cwgrad --C 256 --K 64 --H 56 --k 1 --sweep 1,2,3,4,5,6,7,8,9,11,14,16
} > gpurun_out/r3b/sweep.jsonl 2>&1 || exit 1
echo sweep_ok
CTR_OUT=gpurun_out/r3b/ctr_nt PROBE_ARGS="--op conv --dtype f32 --C 64 --H 56 --k 3 --cfg 104" KFILTER=gemm_nt \
  bash scripts/gpurun/gemm_counters.sh > gpurun_out/r3b/ctr_nt.log 2>&1
CTR_OUT=gpurun_out/r3b/ctr_tn PROBE_ARGS="--op cwgrad --dtype f32 --C 256 --H 14 --k 3 --cfg 7" KFILTER=gemm_tn \
  bash scripts/gpurun/gemm_counters.sh > gpurun_out/r3b/ctr_tn.log 2>&1
echo ctr_done
