#!/bin/bash
# r5c33 (u32x4 staging, no spills): x62 with the B operand pre-split by the binding (cfg family 3): tests + sweep vs family 2
set -u
D=gpurun_out/r5c33
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_x6_gpu.py -k "x62 or split3" > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; tail -15 $D/t.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
S=200001,200002,200003,200004,200005,200006,200007,300001,300002,300003,300004,300005,300006,300007
for sh in "768 3072 16 64" "3072 768 16 64" "768 2304 16 64" "768 768 16 64" "512 2048 7 512" "2048 512 7 512" "64 256 56 512" "256 64 56 512" "1024 256 14 512" "128 512 28 512"; do
  set -- $sh
  timeout -k 10 120 python3 bench/gemm_probe.py --op gemm --dtype f32 --C $1 --K $2 --H $3 --batch $4 --sweep $S >> $D/sweep.jsonl 2>&1 || exit 1
done
for sh in "64 56 64 1" "128 28 128 1" "256 14 256 1" "512 7 512 1" "128 56 128 2" "256 28 256 2" "512 14 512 2" "256 56 512 2"; do
  set -- $sh
  timeout -k 10 120 python3 bench/gemm_probe.py --op conv --dtype f32 --C $1 --H $2 --K $3 --k 3 --stride $4 --batch 512 --sweep 200001,200002,200003,200004,300001,300002,300003,300004 >> $D/conv.jsonl 2>&1 || exit 1
done
for f in sweep conv; do
python3 - <<PY
import json
best = {}
for l in open("$D/$f.jsonl"):
    if not l.startswith("{"): continue
    d = json.loads(l)
    if "us" not in d: print(l.strip()[:200]); continue
    k = (d["C"], d.get("K"), d["H"], d.get("stride"), "x63" if d["cfg"] >= 300000 else "x62")
    best[k] = min(best.get(k, (1e9, 0, 0)), (d["us"], d["cfg"], d["tflops"]))
for k in sorted(best, key=str): print(k, best[k])
PY
done
