#!/bin/bash
# Winograd: pipelined-read vs simple compute, NOLSTORE; PMC counters (C=128 fwd / wgrad)
set -u
D=gpurun_out/s2e
mkdir -p $D
for v in base SIMPLE NOLSTORE; do
  timeout -k 5 60 ./bench/bin/wino_probe_$v 512 20 $v >> $D/probe.jsonl 2> $D/probe_$v.err || { echo "probe $v failed"; exit 1; }
done
echo probes_ok
for op in 0 2; do CTR_OUT=$D/ctr VARIANT=base C=128 OP=$op bash scripts/gpurun/wino_counters.sh || exit 1; done
