#!/bin/bash
# r4 call 30: Winograd grad-weight finalize parallel over the split partials -- Winograd tests, headline, bs32
set -u
D=gpurun_out/r4c30
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_winograd_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -1 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-bf16-phase --ref-batch 0 --json-out $D/head.json > $D/head.log 2>&1
rc=$?; echo head_rc=$rc; python3 -c "import json;d=json.load(open('$D/head.json'));print('head', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --batch-size 32 --steps 40 --warmup 10 --no-bf16-phase --ref-batch 0 --json-out $D/bs32.json > $D/bs32.log 2>&1
rc=$?; echo bs32_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32.json'));print('bs32', d['value'], d['ms_per_step'])"
