#!/bin/bash
# r4 call 17: lazy BN backward (GKSGD_BN_LAZY=1: consumers read dz and x, no bn_bwd_apply pass) re-measured
# on the round-4 kernels -- retune with its keys, replay, and the default for reference
set -u
D=gpurun_out/r4c17
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --no-bf16-phase --ref-batch 0"
show() { python3 -c "import json;d=json.load(open('$D/$1.json'));print('$1', d['value'], d['ms_per_step'])"; }
timeout -k 10 400 $B --json-out $D/default.json > $D/default.log 2>&1
rc=$?; echo default_rc=$rc; show default; [ $rc -eq 0 ] || exit $rc
GKSGD_BN_LAZY=1 GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_SAVE=$D/choices_lazy.json timeout -k 10 700 $B --json-out $D/lazy_tune.json > $D/lazy_tune.log 2>&1
rc=$?; echo lazyt_rc=$rc; show lazy_tune; [ $rc -eq 0 ] || exit $rc
GKSGD_BN_LAZY=1 GKSGD_GEMM_CACHE=$D/choices_lazy.json timeout -k 10 400 $B --json-out $D/lazy.json > $D/lazy.log 2>&1
rc=$?; echo lazy_rc=$rc; show lazy
