#!/bin/bash
# r5c12: bf16x6 NT kernel experiments: base vs bit-slice split (x6e1: VALU cost) vs one product (x6e2: data movement)
set -u
D=gpurun_out/r5c12
mkdir -p $D
export TMPDIR=/tmp
S=100003,100104,100101,100013,100002,100202,101002
for v in base x6e1 x6e2; do
  if [ $v = base ]; then E=""; else E="GKSGD_EXT=variants/$v/_C.so"; fi
  env $E timeout -k 10 120 python3 bench/gemm_probe.py --op gemm --dtype f32 --C 768 --K 3072 --H 16 --batch 64 --sweep $S > $D/bert_$v.jsonl 2>&1 || exit 1
  env $E timeout -k 10 120 python3 bench/gemm_probe.py --op gemm --dtype f32 --C 512 --K 2048 --H 7 --batch 512 --sweep $S > $D/r50_$v.jsonl 2>&1 || exit 1
done
for f in $D/*.jsonl; do echo $f; grep '^{' $f | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('  ', d.get('cfg'), d.get('us'), d.get('tflops'))"; done
