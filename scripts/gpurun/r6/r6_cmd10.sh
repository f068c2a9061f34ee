#!/bin/bash
# r6c10: BN streaming passes -- ReLU-mask cost (fwd_pre vs fwd_pre_norelu) and a torch copy baseline
set -u
D=gpurun_out/r6c10
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python3 bench/bn_probe.py --blocks 1024 --dtype f32 > $D/bn_f32.log 2>&1 || exit 1
timeout -k 10 300 python3 bench/bn_probe.py --blocks 1024 --dtype bf16 > $D/bn_bf16.log 2>&1 || exit 1
cat $D/bn_f32.log $D/bn_bf16.log
