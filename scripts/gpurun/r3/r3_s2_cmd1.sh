#!/bin/bash
# session-2 state check: GPU suite, fp32-headline bench (+bf16 phase), fp32 step profile
set -u
D=gpurun_out/s2a
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D/prof_fp32 -o run -- python3 bench.py --steps 10 --warmup 3 --no-bf16-phase > $D/prof_fp32.log 2>&1
echo prof_rc=$?
