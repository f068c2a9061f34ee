#!/bin/bash
# r4 call 23: Winograd forward with the transform writes spread from xi = 12 -- tests, headline bench
set -u
D=gpurun_out/r4c23
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_winograd_gpu.py tests/test_bn_lazy_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-bf16-phase --ref-batch 0 --json-out $D/head.json > $D/head.log 2>&1
rc=$?; echo head_rc=$rc; python3 -c "import json;d=json.load(open('$D/head.json'));print('head', d['value'], d['ms_per_step'])"
