#!/bin/bash
# full GPU suite, fp32 / bf16 step profiles, GEMM PMC counters
set -u
D=gpurun_out/s2i
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 520 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/prof_fp32 -o run -- python3 bench.py --steps 10 --warmup 3 --no-bf16-phase > $D/prof_fp32.log 2>&1
echo prof_rc=$?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/prof_bf16 -o run -- python3 bench.py --amp bf16 --steps 10 --warmup 3 > $D/prof_bf16.log 2>&1
echo prof16_rc=$?
CTR_D=$D bash scripts/gpurun/r3/r3_counters.sh > $D/ctr.log 2>&1
echo ctr_rc=$?
