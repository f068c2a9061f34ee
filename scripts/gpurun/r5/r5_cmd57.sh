#!/bin/bash
# r5c57: BN streaming-pass workgroup sweep on the round-5 kernels (bench/bn_probe.py), fp32 and bf16
set -u
D=gpurun_out/r5c57
mkdir -p $D
export TMPDIR=/tmp
for dt in f32 bf16; do
  timeout -k 10 300 python3 bench/bn_probe.py --batch 512 --dtype $dt --blocks 768,1024,1536,2048,3072 --json-out $D/bn_$dt.json > $D/bn_$dt.txt 2>&1
  rc=$?; echo bn_${dt}_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/bn_$dt.txt; exit $rc; }
  tail -25 $D/bn_$dt.txt
done
