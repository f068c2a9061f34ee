#!/bin/bash
# r5c4: ResNet-50 bs32 fp32 with batched weight re-layouts (finalize as its own launch again): eager x2,
# without re-layout batching, whole-step graph; kernel profile; then the BERT / compression A/B (r5c3)
set -u
D=gpurun_out/r5c4
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --batch-size 32 --steps 40 --warmup 10 --no-bf16-phase --ref-batch 0"
show() { python3 -c "import json;d=json.load(open('$D/$1.json'));print('$1', d['value'], d['ms_per_step'])"; }
timeout -k 10 300 $B --json-out $D/bs32_eager.json > $D/bs32_eager.log 2>&1
rc=$?; echo eager_rc=$rc; show bs32_eager; [ $rc -eq 0 ] || exit $rc
GKSGD_WEIGHT_PREP=0 timeout -k 10 300 $B --json-out $D/bs32_noprep.json > $D/bs32_noprep.log 2>&1
rc=$?; echo noprep_rc=$rc; show bs32_noprep; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $B --graph --json-out $D/bs32_graph.json > $D/bs32_graph.log 2>&1
rc=$?; echo graph_rc=$rc; show bs32_graph; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $B --json-out $D/bs32_eager2.json > $D/bs32_eager2.log 2>&1
rc=$?; echo eager2_rc=$rc; show bs32_eager2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --batch-size 32 --steps 10 --warmup 5 --no-bf16-phase --ref-batch 0 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker reduce_records_kernel --steps 10 $(find $D/prof -name '*.db' | head -1) $D/prof_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
find $D/prof -name '*.db' -delete
head -14 $D/prof_summary.txt
bash scripts/gpurun/r5/r5_cmd3.sh
