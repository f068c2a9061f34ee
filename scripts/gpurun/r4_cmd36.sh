#!/bin/bash
# r4 call 36: bf16 headline choices -- retune on the final round-4 kernels, then interleaved replay:
# retuned vs committed vs the round-3 bf16 choices
set -u
D=gpurun_out/r4c36
mkdir -p $D
export TMPDIR=/tmp
B="python3 -u bench.py --amp bf16 --steps 20 --warmup 5 --no-bf16-phase --ref-batch 0"
GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_SAVE=$D/choices_bf16.json timeout -k 10 600 $B --json-out $D/retune.json > $D/retune.log 2>&1
rc=$?; echo retune_rc=$rc; python3 -c "import json;d=json.load(open('$D/retune.json'));print('retune', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
for v in new cur r3 new2 cur2 r32; do
  case $v in new*) export GKSGD_GEMM_CACHE=$D/choices_bf16.json ;; r3*) export GKSGD_GEMM_CACHE=tuning/bf16_choices_r3.json ;; *) unset GKSGD_GEMM_CACHE ;; esac
  timeout -k 10 300 $B --json-out $D/$v.json > $D/$v.log 2>&1
  rc=$?; echo ${v}_rc=$rc; python3 -c "import json;d=json.load(open('$D/$v.json'));print('$v', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
done
