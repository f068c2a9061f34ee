#!/bin/bash
# r4 call 3: fp32 attention + fp32 FastLinear tests; fp32 BERT bench + profile; bf16-slowdown profile pair
set -u
D=gpurun_out/r4c3
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_attention_f32_gpu.py tests/test_linear_gpu.py tests/test_attention_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -15 $D/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
GKSGD_GEMM_SAVE=$D/gemm_choices_bert.json timeout -k 10 600 python3 bench.py --model bert --steps 10 --warmup 5 --json-out $D/bert.json > $D/bert.log 2>&1
rc=$?; echo bert_rc=$rc; cat $D/bert.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $D/profb -o prof -- python3 bench.py --model bert --steps 5 --warmup 3 --no-bf16-phase --ref-batch 0 > $D/profb.log 2>&1
rc=$?; echo profb_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker fused_sgd --steps 5 $(find $D/profb -name '*.db' | head -1) $D/bert_f32_summary.txt > $D/sumb.log 2>&1; echo sumb_rc=$?
find $D/profb -name '*.db' -delete
head -16 $D/bert_f32_summary.txt
