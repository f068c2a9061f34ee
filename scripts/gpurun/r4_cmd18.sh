#!/bin/bash
# r4 call 18: Winograd F(2x2,3x3) ablation (drop loads / LDS transform stores /
# epilogue / barriers) on the bs512 shapes, to locate the MFMA idle time
set -u
D=gpurun_out/r4c18
mkdir -p $D
export TMPDIR=/tmp
for v in base NOLOAD NOLSTORE NOBAR NOEPI; do
  timeout -k 5 90 ./bench/pbin/wino_probe_$v 512 20 $v >> $D/probe.jsonl 2> $D/probe_$v.err || { echo "probe $v failed"; exit 1; }
done
echo probes_ok
PROBE_DIR=./bench/pbin CTR_OUT=$D/ctr VARIANT=base C=128 OP=0 bash scripts/gpurun/wino_counters.sh
