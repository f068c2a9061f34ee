#!/bin/bash
# r6c36: ResNet-50 bs512 fp32 / bf16 headline kernel profiles with the grad-weight side stream (default),
# including the GPU wall / busy / concurrent-kernel time per step
set -u
D=gpurun_out/r6c36
mkdir -p $D
export TMPDIR=/tmp
for spec in "fp32 none" "bf16 bf16"; do
  set -- $spec; tag=$1; amp=$2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_$tag -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 5 --amp $amp --model-phases none --no-native-phase --no-bf16-phase --ref-batch 0 --json-out $D/$tag.json > $D/prof_$tag.log 2>&1
  rc=$?; echo prof_${tag}_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/prof_$tag.log; exit $rc; }
  python3 scripts/rocpd_summary.py --marker mc_stats --marker-per-step 1 --steps 10 --title "ResNet-50 bs512 $tag headline, grad-weight side stream (r6c36)" $(find $D/prof_$tag -name '*.db' | head -1) $D/${tag}_summary.csv > $D/sum_$tag.log 2>&1; echo sum_rc=$?
  find $D/prof_$tag -name '*.db' -delete
  head -12 $D/${tag}_summary.csv | cut -c1-200
done
