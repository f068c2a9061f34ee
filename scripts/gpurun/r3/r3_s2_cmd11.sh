#!/bin/bash
# large-tile bf16 GEMM: tests, probe vs hipBLASLt, BERT bench (fresh linear autotune)
set -u
D=gpurun_out/s2m
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 $D/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u bench/big_probe.py > $D/probe.jsonl 2> $D/probe.err
echo probe_rc=$?; cat $D/probe.jsonl
export GKSGD_GEMM_DUMP=$D/tune_dump.json GKSGD_GEMM_SAVE=$D/choices.json
timeout -k 10 400 python -u bench.py --model bert --amp bf16 --steps 10 --warmup 5 > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-200
