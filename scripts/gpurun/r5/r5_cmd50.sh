#!/bin/bash
# r5c50: kernel profile of the bf16 headline (--amp bf16, headline phase only)
set -u
D=gpurun_out/r5c50
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --amp bf16 --steps 10 --warmup 5 --no-native-phase --ref-batch 0 --json-out $D/bench.json > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc
