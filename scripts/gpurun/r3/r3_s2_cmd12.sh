#!/bin/bash
# Winograd pipelined operand reads: tests, probe (new vs prev), fp32 bench
set -u
D=gpurun_out/s2o
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_winograd_gpu.py tests/test_gemm_f32_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 $D/tests.log
[ $rc -eq 0 ] || exit $rc
for v in base prev; do
  timeout -k 5 60 ./bench/bin/wino_probe_$v 512 20 $v >> $D/probe.jsonl 2> $D/probe_$v.err || { echo "probe $v failed"; exit 1; }
done
export GKSGD_GEMM_SAVE=$D/choices.json
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-200
