#!/bin/bash
# Winograd two-stage prefetch: tests, probe (pf2 vs pf1), counters, fp32 bench with choices saved
set -u
D=gpurun_out/s2g
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_winograd_gpu.py > $D/wino_tests.log 2>&1
rc=$?; echo wino_tests_rc=$rc; tail -2 $D/wino_tests.log
[ $rc -eq 0 ] || exit $rc
for v in base pf1; do
  timeout -k 5 60 ./bench/bin/wino_probe_$v 512 20 $v >> $D/probe.jsonl 2> $D/probe_$v.err || { echo "probe $v failed"; exit 1; }
done
CTR_OUT=$D/ctr VARIANT=base C=128 OP=0 bash scripts/gpurun/wino_counters.sh || exit 1
export GKSGD_GEMM_SAVE=$D/choices.json GKSGD_GEMM_DUMP=$D/tune_dump.json
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-300
