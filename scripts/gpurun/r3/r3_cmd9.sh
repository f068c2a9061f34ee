#!/bin/bash
set -u
D=gpurun_out/r3i
mkdir -p $D
timeout -k 10 300 python -u bench/bn_probe.py --dtype f32 --blocks 1024,2048 --json-out $D/bn_f32.json > $D/bn_f32.log 2>&1
echo rc=$?; grep '{' $D/bn_f32.log
