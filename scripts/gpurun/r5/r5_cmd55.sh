#!/bin/bash
# r5c55: headline kernel profile on the rebuilt HEAD (per-kernel comparison against r5c52's
# profiles/r05_resnet50_bs512_fp32_head_kernel_stats.csv: uniform slow-down = box clocks,
# specific kernels = build), GPU clocks read before / after, FCN-5 first-phase check
set -u
D=gpurun_out/r5c55
mkdir -p $D
export TMPDIR=/tmp
(rocm-smi --showclocks --showpower --showtemp > $D/smi_before.txt 2>&1 || true)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 5 --no-native-phase --no-bf16-phase --ref-batch 0 --json-out $D/prof_bench.json > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/prof.log; exit $rc; }
(rocm-smi --showclocks --showpower --showtemp > $D/smi_after.txt 2>&1 || true)
python3 scripts/rocpd_summary.py --marker select_kernel --steps 10 --title "ResNet-50 bs512 fp32 headline, rebuilt HEAD (r5c55)" $(find $D/prof -name '*.db' | head -1) $D/head_summary.csv > $D/sum.log 2>&1; echo sum_rc=$?
find $D/prof -name '*.db' -delete
head -14 $D/head_summary.csv
python3 -c "
import json;d=json.load(open('$D/prof_bench.json'));print({k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step')})"
timeout -k 10 300 python3 bench.py --model fcn5net --steps 50 --warmup 200 --no-bf16-phase --ref-batch 0 --json-out $D/fcn5_w200.json > $D/fcn5.log 2>&1
rc=$?; echo fcn5_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json;d=json.load(open('$D/fcn5_w200.json'));print({k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step')})"
