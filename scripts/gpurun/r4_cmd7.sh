#!/bin/bash
# r4 call 7: bf16 NT issue order restored (fp32 keeps the spread), count / select two-tile rings --
# tests, compression kernels, headline + bf16 phase, ResNet-50 bs32 old vs retuned choices
set -u
D=gpurun_out/r4c7
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_conv1x1_gpu.py tests/test_bnlink_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench/kernels.py --only compress,round2 --json-out $D/kernels.json > $D/kernels.log 2>&1
rc=$?; echo kernels_rc=$rc; grep -i compress $D/kernels.log
show() { python3 -c "import json;d=json.load(open('$D/$1.json'));print('$1', d['value'], d['ms_per_step'], d.get('bf16_value'), d.get('bf16_ms_per_step'))"; }
timeout -k 10 400 python3 bench.py --ref-batch 0 --json-out $D/head.json > $D/head.log 2>&1
rc=$?; echo head_rc=$rc; show head; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --batch-size 32 --steps 40 --warmup 10 --no-bf16-phase --ref-batch 0"
timeout -k 10 300 $B --json-out $D/bs32_old.json > $D/bs32_old.log 2>&1
rc=$?; echo old_rc=$rc; show bs32_old; [ $rc -eq 0 ] || exit $rc
GKSGD_GEMM_CACHE=tuning/choices_bs32_r4c6.json timeout -k 10 300 $B --json-out $D/bs32_new.json > $D/bs32_new.log 2>&1
rc=$?; echo new_rc=$rc; show bs32_new; [ $rc -eq 0 ] || exit $rc
GKSGD_GEMM_CACHE=tuning/choices_bs32_r4c6.json timeout -k 10 300 $B --graph --json-out $D/bs32_new_graph.json > $D/bs32_new_graph.log 2>&1
rc=$?; echo graph_rc=$rc; show bs32_new_graph
