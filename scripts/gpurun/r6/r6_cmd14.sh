#!/bin/bash
# r6c14: bf16x6 stem grad-weight staged split interleaved with the MFMAs -- stem tests + probe (occupancy 1 / 2, bs128 / bs512)
set -u
D=gpurun_out/r6c14
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_stem_gpu.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
PYTHONPATH=. timeout -k 10 120 python3 bench/stem_x6_probe.py > $D/probe1.json 2> $D/probe1.err || exit 1

PYTHONPATH=. N=512 timeout -k 10 120 python3 bench/stem_x6_probe.py > $D/probe512.json 2> $D/probe512.err || exit 1
cat $D/probe1.json $D/probe512.json
