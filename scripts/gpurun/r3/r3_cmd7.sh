#!/bin/bash
set -u
D=gpurun_out/r3g
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_e2e_gpu.py \
  tests/test_conv1x1_gpu.py tests/test_bnlink_gpu.py tests/test_graph_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -15 $D/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 $D/bench.log
[ $rc -eq 0 ] || exit $rc
GKSGD_WGRAD_STREAM=0 timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $D/bench_nostream.json > $D/bench_nostream.log 2>&1
echo nostream_rc=$?
