#!/bin/bash
# r6c44: LSTM bs128 fp32 ordered kernel sequence of one step (what the 19 direct_copy kernels per step are)
set -u
D=gpurun_out/r6c44
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $D/prof -o run -- python3 bench.py --gpus 1 --steps 4 --warmup 3 --model lstm --model-phases none --no-native-phase --no-bf16-phase --ref-batch 0 --json-out $D/lstm.json > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/prof.log; exit $rc; }
python3 scripts/rocpd_summary.py --marker mc_stats --steps 4 --sequence $D/seq.csv --title "lstm seq" $(find $D/prof -name '*.db' | head -1) $D/sum.csv > /dev/null 2>&1; echo sum_rc=$?
find $D/prof -name '*.db' -delete
grep -n -B2 -A2 "direct_copy\|copyBuffer\|FillFunctor" $D/seq.csv | cut -c1-160 | head -120
