#!/bin/bash
# r4 call 20: forward Winograd transform slot (x8 = xi 8, x12, x14) vs burst base
set -u
D=gpurun_out/r4c20
mkdir -p $D
export TMPDIR=/tmp
for v in base x8 x12 x14 base x8 x12 x14; do
  timeout -k 5 90 ./bench/pbin/wino_probe_$v 512 20 $v 0 0 >> $D/probe.jsonl 2> $D/probe_$v.err || { echo "probe $v failed"; exit 1; }
done
echo probes_ok
