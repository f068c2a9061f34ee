#!/bin/bash
# round-end rehearsal: full GPU test suite, smoke(), headline bench (fp32 + bf16 phase)
set -u
D=gpurun_out/final
mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -2 $D/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
echo done
