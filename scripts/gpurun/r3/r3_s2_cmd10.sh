#!/bin/bash
# BERT bench with the autotune dump (own GEMM vs hipBLASLt timings per linear shape)
set -u
D=gpurun_out/s2l
mkdir -p $D
export TMPDIR=/tmp GKSGD_GEMM_DUMP=$D/tune_dump.json GKSGD_GEMM_RETUNE=1
timeout -k 10 400 python -u bench.py --model bert --amp bf16 --steps 10 --warmup 5 > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-300
