#!/bin/bash
# r5c58: reference-batch (bs32) fp32 kernel profile at the final HEAD (whole-step HIP graph, as the
# bench's ref_bs32 phase), kernel summary of the last 10 steps
set -u
D=gpurun_out/r5c58
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 bench.py --gpus 1 --batch-size 32 --graph --steps 20 --warmup 10 --no-native-phase --no-bf16-phase --ref-batch 0 --json-out $D/bs32.json > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/prof.log; exit $rc; }
python3 scripts/rocpd_summary.py --marker select_kernel --steps 10 --title "ResNet-50 bs32 fp32 (reference batch), whole-step HIP graph, final round-5 HEAD (r5c58)" $(find $D/prof -name '*.db' | head -1) $D/bs32_summary.csv > $D/sum.log 2>&1; echo sum_rc=$?
find $D/prof -name '*.db' -delete
head -16 $D/bs32_summary.csv
grep -E "finalize" $D/bs32_summary.csv | cut -c1-120
python3 -c "
import json;d=json.load(open('$D/bs32.json'));print({k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step')})"
