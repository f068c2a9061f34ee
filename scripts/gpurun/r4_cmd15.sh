#!/bin/bash
# r4 call 15: hand-off A/B in whole steps (launch vs last-block) -- BERT fp32 (14 overlapped buckets)
# and the default bench.py line (ResNet-50 headline + bf16 + bs32 phases)
set -u
D=gpurun_out/r4c15
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --model bert --no-bf16-phase --ref-batch 0 --steps 8 --warmup 4"
show() { python3 -c "import json;d=json.load(open('$D/$1.json'));print('$1', d['value'], d['ms_per_step'], d.get('bf16_value'), d.get('ref_bs32_value'), d.get('ref_bs32_dense_value'))"; }
timeout -k 10 400 $B --json-out $D/bert_launch.json > $D/bert_launch.log 2>&1
rc=$?; echo bl_rc=$rc; show bert_launch; [ $rc -eq 0 ] || exit $rc
GKSGD_HANDOFF=lastblock timeout -k 10 400 $B --json-out $D/bert_last.json > $D/bert_last.log 2>&1
rc=$?; echo bla_rc=$rc; show bert_last; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py --json-out $D/default_launch.json > $D/default_launch.log 2>&1
rc=$?; echo dl_rc=$rc; show default_launch; [ $rc -eq 0 ] || exit $rc
GKSGD_HANDOFF=lastblock timeout -k 10 500 python3 bench.py --json-out $D/default_last.json > $D/default_last.log 2>&1
rc=$?; echo dla_rc=$rc; show default_last
