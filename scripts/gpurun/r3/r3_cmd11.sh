#!/bin/bash
set -u
D=gpurun_out/r3l
mkdir -p $D
for v in base ntst ntld ntboth; do
  if [ $v = base ]; then unset GKSGD_EXT; else export GKSGD_EXT=variants/$v/_C.so; fi
  timeout -k 10 200 python -u bench/bn_probe.py --dtype f32 --blocks 1024 > $D/bn_$v.log 2>&1
  echo "$v rc=$?"
done
unset GKSGD_EXT
timeout -k 10 200 python -u bench/bn_probe.py --dtype bf16 --blocks 1024 > $D/bn16_base.log 2>&1
GKSGD_EXT=variants/ntboth/_C.so timeout -k 10 200 python -u bench/bn_probe.py --dtype bf16 --blocks 1024 > $D/bn16_ntboth.log 2>&1
echo done
