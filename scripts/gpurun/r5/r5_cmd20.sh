#!/bin/bash
# r5c20: SLP-vectorized (v_pk_add_f32) split vs scalar subtractions (noslp: -fno-slp-vectorize): GEMM sweeps (x6 and native) + fp32 headline
set -u
D=gpurun_out/r5c20
mkdir -p $D
export TMPDIR=/tmp
S=100104,100101,100013,100003,100202,104,1002,3,13
for v in base noslp; do
  if [ $v = base ]; then E=""; else E="GKSGD_EXT=variants/$v/_C.so"; fi
  for sh in "768 3072 16 64" "3072 768 16 64" "768 2304 16 64" "512 2048 7 512" "64 256 56 512" "1024 256 14 512"; do
    set -- $sh
    env $E timeout -k 10 120 python3 bench/gemm_probe.py --op gemm --dtype f32 --C $1 --K $2 --H $3 --batch $4 --sweep $S >> $D/$v.jsonl 2>&1 || exit 1
  done
done
python3 - <<PY
import json
for v in ("base", "noslp"):
    best = {}
    for l in open("$D/%s.jsonl" % v):
        if not l.startswith("{"): continue
        d = json.loads(l); k = (d["C"], d["K"], d["H"], "x6" if d["cfg"] >= 100000 else "f32")
        best[k] = min(best.get(k, (1e9, 0)), (d["us"], d["cfg"]))
    print(v, sorted(best.items()))
PY
for v in base noslp; do
  if [ $v = base ]; then E=""; else E="GKSGD_EXT=variants/$v/_C.so"; fi
  env $E timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-bf16-phase --ref-batch 0 --json-out $D/b_$v.json > $D/b_$v.log 2>&1 || exit 1
  python3 -c "import json;d=json.load(open('$D/b_$v.json'));print('$v', d['value'], d['ms_per_step'])"
done
