#!/bin/bash
# r4 call 32: PMC counters of the final Winograd kernels (C = K = 128, 28 x 28, bs512): forward and grad-weight
set -u
D=gpurun_out/r4c32
mkdir -p $D
export TMPDIR=/tmp
PROBE_DIR=./variants/probe CTR_OUT=$D/ctr VARIANT=base C=128 OP=0 bash scripts/gpurun/wino_counters.sh
PROBE_DIR=./variants/probe CTR_OUT=$D/ctr VARIANT=base C=128 OP=2 bash scripts/gpurun/wino_counters.sh
python3 scripts/wino_ctr_summary.py $D/ctr > $D/summary.txt 2>&1; cat $D/summary.txt
