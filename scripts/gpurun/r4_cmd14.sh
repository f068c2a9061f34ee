#!/bin/bash
# r4 call 14: fp32 fused add + LayerNorm -- tests; BERT fp32 with it vs PyTorch LN (same tuning cache);
# BERT fp32 kernel profile
set -u
D=gpurun_out/r4c14
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ln_gpu.py tests/test_attention_f32_gpu.py > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/r4c8/choices_bert.json $D/choices_bert.json 2>/dev/null || true
B="python3 bench.py --model bert --no-bf16-phase --ref-batch 0 --steps 8 --warmup 4"
show() { python3 -c "import json;d=json.load(open('$D/$1.json'));print('$1', d['value'], d['ms_per_step'], d['config']['buckets'])"; }
timeout -k 10 400 $B --json-out $D/bert_ln.json > $D/bert_ln.log 2>&1
rc=$?; echo ln_rc=$rc; show bert_ln; [ $rc -eq 0 ] || exit $rc
GKSGD_LN_F32=0 timeout -k 10 400 $B --json-out $D/bert_noln.json > $D/bert_noln.log 2>&1
rc=$?; echo noln_rc=$rc; show bert_noln; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --model bert --no-bf16-phase --ref-batch 0 --steps 5 --warmup 3 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker attn_f32_fwd --marker-per-step 12 --steps 5 $(find $D/prof -name '*.db' | head -1) $D/bert_f32_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
head -14 $D/bert_f32_summary.txt
