#!/bin/bash
# r5c11: bf16x6 GEMM tests; ResNet-50 bs512 fp32 headline, native vs bf16x6 GEMM candidates
# (tuned in the warm-up; x6 choices saved)
set -u
D=gpurun_out/r5c11
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_x6_gpu.py > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; tail -30 $D/t.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 20 --warmup 5 --no-bf16-phase --ref-batch 0"
timeout -k 10 400 $B --f32-matmul native --json-out $D/native.json > $D/native.log 2>&1
rc=$?; echo native_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/native.log; exit $rc; }
GKSGD_GEMM_SAVE=$D/choices_x6.json GKSGD_GEMM_DUMP=$D/dump_x6.json timeout -k 10 600 $B --f32-matmul bf16x6 --json-out $D/x6.json > $D/x6.log 2>&1
rc=$?; echo x6_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/x6.log; exit $rc; }
python3 -c "
import json
for n in ('native','x6'):
    d=json.load(open('$D/%s.json'%n)); print(n, d['value'], d['ms_per_step'], d['config'].get('f32_matmul'))"
