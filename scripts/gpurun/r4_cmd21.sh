#!/bin/bash
# r4 call 21: forward Winograd staggered transform slots (wave group 0 / 1): s4_12, s12_12 vs x12 and base
set -u
D=gpurun_out/r4c21
mkdir -p $D
export TMPDIR=/tmp
for v in base x12 s4_12 s12_12 base x12 s4_12 s12_12; do
  timeout -k 5 90 ./bench/pbin/wino_probe_$v 512 20 $v 0 0 >> $D/probe.jsonl 2> $D/probe_$v.err || { echo "probe $v failed"; exit 1; }
  timeout -k 5 90 ./bench/pbin/wino_probe_$v 512 20 $v 0 1 >> $D/probe.jsonl 2>> $D/probe_$v.err || { echo "probe $v failed"; exit 1; }
done
echo probes_ok
