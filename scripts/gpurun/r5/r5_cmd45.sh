#!/bin/bash
# r5c45: x62 gather with 32-bit pixel offsets + packed tap masks (fewer spills): x62 GPU tests + 3x3 conv sweep
set -u
D=gpurun_out/r5c45
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_x6_gpu.py -k "x62 or split3" > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 $D/t.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for sh in "64 56 64 1" "128 28 128 1" "256 14 256 1" "512 7 512 1" "128 56 128 2" "256 28 256 2" "512 14 512 2" "256 56 512 2"; do
  set -- $sh
  timeout -k 10 120 python3 bench/gemm_probe.py --op conv --dtype f32 --C $1 --H $2 --K $3 --k 3 --stride $4 --batch 512 --sweep 200001,200002,200003,200004 >> $D/conv.jsonl 2>&1 || exit 1
done
python3 - <<PY
import json
for l in open("$D/conv.jsonl"):
    if not l.startswith("{"): continue
    d = json.loads(l)
    if "us" not in d: print(l.strip()[:200]); continue
    print(d["C"], d["H"], d["stride"], d["cfg"], d["us"], d["tflops"])
PY
