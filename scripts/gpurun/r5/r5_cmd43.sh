#!/bin/bash
# r5c43: x62 BN-backward epilogue without spills (no bias registers, one fragment of operands at a time):
# x62 GPU tests + BNB grad-input sweep, bf16x6 LDS-DMA (family 1) vs register-staged (2, 3)
set -u
D=gpurun_out/r5c43
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_x6_gpu.py -k "x62 or split3" > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 $D/t.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
S=100001,100002,100003,100004,100005,100006,100007,100101,100102,100103,100104,100105,100106,100107,200001,200002,200003,200004,200005,200006,200007,300001,300002,300003,300004,300005,300006,300007
for sh in "256 64 56 512" "64 256 56 512" "512 128 28 512" "128 512 28 512" "1024 256 14 512" "256 1024 14 512" "2048 512 7 512" "512 2048 7 512"; do
  set -- $sh
  timeout -k 10 120 python3 bench/gemm_probe.py --op gemm_bnb --dtype f32 --C $1 --K $2 --H $3 --batch $4 --sweep $S >> $D/sweep.jsonl 2>&1 || exit 1
done
python3 - <<PY
import json
best = {}
for l in open("$D/sweep.jsonl"):
    if not l.startswith("{"): continue
    d = json.loads(l)
    if "us" not in d: print(l.strip()[:200]); continue
    fam = d["cfg"] // 100000
    k = (d["C"], d["K"], d["H"], "x6" if fam == 1 else ("x62" if fam == 2 else "x63"))
    best[k] = min(best.get(k, (1e9, 0, 0)), (d["us"], d["cfg"], d["tflops"]))
for k in sorted(best, key=str): print(k, best[k])
PY
