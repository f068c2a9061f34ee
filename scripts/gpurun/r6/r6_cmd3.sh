#!/bin/bash
# r6c3: new GPU tests (sync-timeout recovery, bench 2-rank with k_cap = k),
# then kernel profiles of the secondary BASELINE models at the headline
# precision (fp32): VGG-16 CIFAR bs512, LSTM PTB bs128, BERT-base seq512 bs32
set -u
D=gpurun_out/r6c3
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_sync_recovery_gpu.py tests/test_bench_gpu.py -x -v --timeout 600 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -8 $D/tests.log; [ $rc -eq 0 ] || exit $rc
for spec in "vgg16 1" "lstm 1" "bert 14"; do
  set -- $spec; m=$1; nb=$2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_$m -o run -- python3 bench.py --gpus 1 --model $m --steps 10 --warmup 5 --model-phases none --no-native-phase --no-bf16-phase --ref-batch 0 --json-out $D/$m.json > $D/prof_$m.log 2>&1
  rc=$?; echo prof_${m}_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/prof_$m.log; exit $rc; }
  python3 scripts/rocpd_summary.py --marker mc_stats --marker-per-step $nb --steps 10 --title "$m fp32 (bench.py --model $m, headline precision), round-6 HEAD (r6c3)" $(find $D/prof_$m -name '*.db' | head -1) $D/${m}_summary.csv > $D/sum_$m.log 2>&1; echo sum_rc=$?
  find $D/prof_$m -name '*.db' -delete
  head -14 $D/${m}_summary.csv | cut -c1-160
done
