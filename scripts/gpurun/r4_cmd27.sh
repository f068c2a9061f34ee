#!/bin/bash
# r4 call 27: ResNet-50 bs32 fp32 (reference batch) on the final round-4 build: eager and graphed bench lines,
# kernel profile
set -u
D=gpurun_out/r4c27
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --batch-size 32 --steps 40 --warmup 10 --no-bf16-phase --ref-batch 0"
timeout -k 10 300 $B --json-out $D/bs32_eager.json > $D/bs32_eager.log 2>&1
rc=$?; echo eager_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32_eager.json'));print('eager', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $B --graph --json-out $D/bs32_graph.json > $D/bs32_graph.log 2>&1
rc=$?; echo graph_rc=$rc; python3 -c "import json;d=json.load(open('$D/bs32_graph.json'));print('graph', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --batch-size 32 --steps 10 --warmup 5 --no-bf16-phase --ref-batch 0 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker reduce_records_kernel --steps 10 $(find $D/prof -name '*.db' | head -1) $D/prof_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
head -14 $D/prof_summary.txt
