#!/bin/bash
# r5c15: bf16x6 NT: software-pipelined loop (sched_group_barrier interleave) vs the first form (x6old)
set -u
D=gpurun_out/r5c15
mkdir -p $D
export TMPDIR=/tmp
true

S=100104,100101,100013,100003,100202,101002
for v in base x6old; do
  if [ $v = base ]; then E=""; else E="GKSGD_EXT=variants/$v/_C.so"; fi
  for sh in "768 3072 16 64" "3072 768 16 64" "512 2048 7 512" "64 256 56 512" "256 64 56 512"; do
    set -- $sh
    env $E timeout -k 10 120 python3 bench/gemm_probe.py --op gemm --dtype f32 --C $1 --K $2 --H $3 --batch $4 --sweep $S >> $D/$v.jsonl 2>&1 || exit 1
  done
done
python3 - <<PY
import json
for v in ("base", "x6old"):
    best = {}
    for l in open("$D/%s.jsonl" % v):
        if not l.startswith("{"): continue
        d = json.loads(l); k = (d["C"], d["K"], d["H"])
        best[k] = min(best.get(k, (1e9, 0)), (d["us"], d["cfg"]))
    print(v, best)
PY
