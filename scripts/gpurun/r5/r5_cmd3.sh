#!/bin/bash
# r5c3: BERT fp32 (config 5): in-grid hand-offs for the buckets that overlap the backward vs separate
# launches; BERT kernel profile; compression pipeline on the 25.6 M bucket, both hand-off forms
set -u
D=gpurun_out/r5c3
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --model bert --no-bf16-phase --ref-batch 0 --steps 8 --warmup 4"
show() { python3 -c "import json;d=json.load(open('$D/$1.json'));print('$1', d['value'], d['ms_per_step'], d['config']['buckets'], d.get('exposed_comm_ms'))"; }
timeout -k 10 400 $B --json-out $D/bert_lastblock.json > $D/bert_lastblock.log 2>&1
rc=$?; echo lb_rc=$rc; show bert_lastblock; [ $rc -eq 0 ] || exit $rc
GKSGD_OVERLAP_HANDOFF=launch timeout -k 10 400 $B --json-out $D/bert_launch.json > $D/bert_launch.log 2>&1
rc=$?; echo launch_rc=$rc; show bert_launch; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 $B --json-out $D/bert_lastblock2.json > $D/bert_lastblock2.log 2>&1
rc=$?; echo lb2_rc=$rc; show bert_lastblock2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --model bert --no-bf16-phase --ref-batch 0 --steps 5 --warmup 3 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker attn_f32_fwd --marker-per-step 12 --steps 5 $(find $D/prof -name '*.db' | head -1) $D/bert_f32_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
find $D/prof -name '*.db' -delete
head -14 $D/bert_f32_summary.txt
timeout -k 10 300 python3 bench/kernels.py --only round2 --json-out $D/k_launch.json > $D/k_launch.log 2>&1
rc=$?; echo klaunch_rc=$rc; grep -i compress $D/k_launch.log; [ $rc -eq 0 ] || exit $rc
GKSGD_HANDOFF=lastblock timeout -k 10 300 python3 bench/kernels.py --only round2 --json-out $D/k_last.json > $D/k_last.log 2>&1
rc=$?; echo klast_rc=$rc; grep -i compress $D/k_last.log
