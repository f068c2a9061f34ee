#!/bin/bash
# r5c30: register-staged bf16x6 row GEMMs  conflict-free LDS swizzle: tests + sweep
set -u
D=gpurun_out/r5c30
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_x6_gpu.py > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; tail -15 $D/t.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
S=100104,100101,100013,100003,100202,200001,200002,200003,200004,200005,200006,200007
for sh in "768 3072 16 64" "3072 768 16 64" "768 2304 16 64" "768 768 16 64" "512 2048 7 512" "2048 512 7 512" "64 256 56 512" "256 64 56 512" "1024 256 14 512" "128 512 28 512"; do
  set -- $sh
  timeout -k 10 120 python3 bench/gemm_probe.py --op gemm --dtype f32 --C $1 --K $2 --H $3 --batch $4 --sweep $S >> $D/sweep.jsonl 2>&1 || exit 1
done
for sh in "64 56 64 1" "128 28 128 1" "256 14 256 1" "512 7 512 1" "128 56 128 2" "256 28 256 2" "512 14 512 2" "256 56 512 2"; do
  set -- $sh
  timeout -k 10 120 python3 bench/gemm_probe.py --op conv --dtype f32 --C $1 --H $2 --K $3 --k 3 --stride $4 --batch 512 --sweep 100104,100101,100013,100003,100202,200001,200002,200003,200004 >> $D/conv.jsonl 2>&1 || exit 1
done
python3 - <<PY2
import json
best = {}
for l in open("$D/conv.jsonl"):
    if not l.startswith("{"): continue
    d = json.loads(l)
    if "us" not in d: print(l.strip()[:200]); continue
    k = (d["C"], d["H"], d["stride"], "x62" if d["cfg"] >= 200000 else "x6")
    best[k] = min(best.get(k, (1e9, 0, 0)), (d["us"], d["cfg"], d["tflops"]))
for k in sorted(best): print(k, best[k])
PY2
python3 - <<PY
import json
best = {}
for l in open("$D/sweep.jsonl"):
    if not l.startswith("{"): continue
    d = json.loads(l)
    if "us" not in d: print(l.strip()[:200]); continue
    k = (d["C"], d["K"], d["H"], ("x62pf2" if (d["cfg"] // 10) % 10 == 1 else "x62") if d["cfg"] >= 200000 else "x6")
    best[k] = min(best.get(k, (1e9, 0, 0)), (d["us"], d["cfg"], d["tflops"]))
for k in sorted(best): print(k, best[k])
PY


