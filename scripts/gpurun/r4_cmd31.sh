#!/bin/bash
# r4 call 31: same-box A/B, Winograd grad-weight finalize parallel over splits (new) vs HEAD (variants/old)
set -u
export TMPDIR=/tmp
AB_OUT=gpurun_out/r4c31 AB_CUT=120 AB_CMDS="python3 bench.py --steps 20 --warmup 5 --no-bf16-phase --ref-batch 0" bash scripts/gpurun/ab.sh
