#!/bin/bash
# r5c27: register-staged bf16x6 grad-weight (TN x62): tests + sweep vs the LDS-DMA bf16x6 TN kernels
set -u
D=gpurun_out/r5c27
mkdir -p $D
export TMPDIR=/tmp
true

S=100004,100007,100014,100015,100016,100008,100005,200001,200002,200003,200004,200005,200006,200007,200008
for sh in "768 3072 16 64" "3072 768 16 64" "768 768 16 64" "512 2048 7 512" "64 256 56 512" "256 64 56 512" "1024 256 14 512"; do
  set -- $sh
  # lwgrad: W[K, C] += G[M, K]^T X[M, C] with M = batch * H
  timeout -k 10 120 python3 bench/gemm_probe.py --op lwgrad --dtype f32 --C $1 --K $2 --H $(( $3 * $3 )) --batch $4 --sweep $S >> $D/sweep.jsonl 2>&1 || exit 1
done
python3 - <<PY
import json
best = {}
for l in open("$D/sweep.jsonl"):
    if not l.startswith("{"): continue
    d = json.loads(l)
    if "us" not in d: print(l.strip()[:200]); continue
    k = (d["C"], d["K"], d["H"], "x62" if d["cfg"] >= 200000 else "x6")
    best[k] = min(best.get(k, (1e9, 0, 0)), (d["us"], d["cfg"], d["tflops"]))
for k in sorted(best): print(k, best[k])
PY
