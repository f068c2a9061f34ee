#!/bin/bash
# fp32 headline bench with the lazy BN backward (+ a GKSGD_BN_LAZY=0 comparison) and its rocprof profile
set -u
D=gpurun_out/r3f
mkdir -p $D
export GKSGD_GEMM_SAVE=$D/choices.json GKSGD_GEMM_DUMP=$D/tune_dump.json
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench_fp32.json > $D/bench_fp32.log 2>&1
rc=$?; echo bench_rc=$rc; tail -2 $D/bench_fp32.log
[ $rc -eq 0 ] || exit $rc
unset GKSGD_GEMM_SAVE GKSGD_GEMM_DUMP
GKSGD_BN_LAZY=0 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-bf16-phase --json-out $D/bench_fp32_nolazy.json > $D/bench_fp32_nolazy.log 2>&1
rc=$?; echo nolazy_rc=$rc
[ $rc -eq 0 ] || exit $rc
export GKSGD_GEMM_CACHE=$PWD/$D/choices.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof_fp32 -o run -- python bench.py --steps 10 --warmup 3 --no-bf16-phase > $D/prof_fp32.log 2>&1
echo prof_rc=$?
