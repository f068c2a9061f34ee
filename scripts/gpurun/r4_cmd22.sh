#!/bin/bash
# r4 call 22: forward Winograd, xi = 15 MFMAs deferred across the stage barrier (d1) vs not (d0)
set -u
D=gpurun_out/r4c22
mkdir -p $D
export TMPDIR=/tmp
for v in d0 d1 d0 d1; do
  timeout -k 5 90 ./bench/pbin/wino_probe_$v 512 20 $v 0 0 >> $D/probe.jsonl 2> $D/probe_$v.err || { echo "probe $v failed"; exit 1; }
  timeout -k 5 90 ./bench/pbin/wino_probe_$v 512 20 $v 0 1 >> $D/probe.jsonl 2>> $D/probe_$v.err || { echo "probe $v failed"; exit 1; }
done
echo probes_ok
