#!/bin/bash
# r5c42: kernel profile of the round-5 HEAD fp32 headline (headline phase only) and BERT fp32
set -u
D=gpurun_out/r5c42
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --steps 10 --warmup 5 --no-bf16-phase --no-native-phase --ref-batch 0 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $D/bprof -o prof -- python3 bench.py --model bert --steps 10 --warmup 3 --no-bf16-phase --no-native-phase > $D/bprof.log 2>&1
rc=$?; echo bprof_rc=$rc
