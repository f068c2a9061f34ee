#!/bin/bash
# r4 call 9: sign-bit candidate counting (count kernel), bf16 NT fragment schedule of round 3 --
# tests, compression kernels (+ profile), headline with the bf16 phase
set -u
D=gpurun_out/r4c9
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels2_gpu.py tests/test_gemm_gpu.py tests/test_conv1x1_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/kernels.py --only compress,round2 --json-out $D/kernels.json > $D/kernels.log 2>&1
rc=$?; echo kernels_rc=$rc; grep -i compress $D/kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d $D/profk -o profk -- python3 bench/kernels.py --only round2 > $D/profk.log 2>&1
rc=$?; echo profk_rc=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --ref-batch 0 --json-out $D/head.json > $D/head.log 2>&1
rc=$?; echo head_rc=$rc; python3 -c "import json;d=json.load(open('$D/head.json'));print('head', d['value'], d['ms_per_step'], d.get('bf16_value'), d.get('bf16_ms_per_step'))"
