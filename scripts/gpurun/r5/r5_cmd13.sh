#!/bin/bash
# r5c13: bf16x6 NT with 128x64 wave tiles (cfg 5-7) vs 64x64
set -u
D=gpurun_out/r5c13
mkdir -p $D
export TMPDIR=/tmp
S=100104,100101,100013,100202,100005,100006,100007,100105,100106,100107
timeout -k 10 120 python3 bench/gemm_probe.py --op gemm --dtype f32 --C 768 --K 3072 --H 16 --batch 64 --sweep $S > $D/bert.jsonl 2>&1 || exit 1
timeout -k 10 120 python3 bench/gemm_probe.py --op gemm --dtype f32 --C 3072 --K 768 --H 16 --batch 64 --sweep $S > $D/bert2.jsonl 2>&1 || exit 1
timeout -k 10 120 python3 bench/gemm_probe.py --op gemm --dtype f32 --C 512 --K 2048 --H 7 --batch 512 --sweep $S > $D/r50.jsonl 2>&1 || exit 1
timeout -k 10 120 python3 bench/gemm_probe.py --op gemm --dtype f32 --C 64 --K 256 --H 56 --batch 512 --sweep $S > $D/r50b.jsonl 2>&1 || exit 1
for f in $D/*.jsonl; do echo $f; grep '^{' $f | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('  ', d.get('cfg'), d.get('us'), d.get('tflops'), d.get('error','')[:80])"; done
