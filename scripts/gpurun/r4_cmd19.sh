#!/bin/bash
# r4 call 19: Winograd LDS transform writes spread over the xi slots (spread)
# vs the burst form (base, r4c18 binary), bs512 shapes
set -u
D=gpurun_out/r4c19
mkdir -p $D
export TMPDIR=/tmp
for v in base spread base spread; do
  timeout -k 5 90 ./bench/pbin/wino_probe_$v 512 20 $v >> $D/probe.jsonl 2> $D/probe_$v.err || { echo "probe $v failed"; exit 1; }
done
echo probes_ok
