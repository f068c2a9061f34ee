#!/bin/bash
# r4 call 37: bs32 fp32 choices -- retune on the final round-4 kernels, then interleaved replay: retuned vs committed
set -u
D=gpurun_out/r4c37
mkdir -p $D
export TMPDIR=/tmp
B="python3 -u bench.py --batch-size 32 --steps 40 --warmup 10 --no-bf16-phase --ref-batch 0"
GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_SAVE=$D/choices_bs32.json timeout -k 10 600 $B --json-out $D/retune.json > $D/retune.log 2>&1
rc=$?; echo retune_rc=$rc; python3 -c "import json;d=json.load(open('$D/retune.json'));print('retune', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
for v in new cur new2 cur2; do
  case $v in new*) export GKSGD_GEMM_CACHE=$D/choices_bs32.json ;; *) unset GKSGD_GEMM_CACHE ;; esac
  timeout -k 10 300 $B --json-out $D/$v.json > $D/$v.log 2>&1
  rc=$?; echo ${v}_rc=$rc; python3 -c "import json;d=json.load(open('$D/$v.json'));print('$v', d['value'], d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
done
