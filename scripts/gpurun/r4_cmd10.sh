#!/bin/bash
# r4 call 10: batched device-coherent hand-off loads (decide / finalize / radix) -- compression
# tests + per-kernel timeline; bf16 with the round-3 bf16 tuning choices vs current
set -u
D=gpurun_out/r4c10
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels2_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/kernels.py --only compress,round2 --json-out $D/kernels.json > $D/kernels.log 2>&1
rc=$?; echo kernels_rc=$rc; grep -i compress $D/kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d $D/profk -o profk -- python3 bench/kernels.py --only round2 > $D/profk.log 2>&1
rc=$?; echo profk_rc=$rc; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --ref-batch 0 --amp bf16 --no-bf16-phase"
timeout -k 10 300 $B --json-out $D/bf16_cur.json > $D/bf16_cur.log 2>&1
rc=$?; echo cur_rc=$rc; python3 -c "import json;d=json.load(open('$D/bf16_cur.json'));print('bf16 cur', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
GKSGD_GEMM_CACHE=tuning/bf16_choices_r3.json timeout -k 10 300 $B --json-out $D/bf16_r3.json > $D/bf16_r3.log 2>&1
rc=$?; echo r3_rc=$rc; python3 -c "import json;d=json.load(open('$D/bf16_r3.json'));print('bf16 r3choices', d['value'], d['ms_per_step'])"
