#!/bin/bash
# r5c48: x62 A-fragment prefetch (GK_X62_APF, 256-thread tiles only): same-box sweep vs variants/old (APF=0)
set -u
D=gpurun_out/r5c48
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_x6_gpu.py -k "x62" > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 $D/t.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
S=200001,200004,200005,200006,200007,200002,200003
for v in new old; do
  if [ $v = old ]; then export GKSGD_EXT=variants/old/_C.so; else unset GKSGD_EXT; fi
  for sh in "768 3072 16 64" "3072 768 16 64" "768 2304 16 64" "768 768 16 64" "512 2048 7 512" "2048 512 7 512" "64 256 56 512" "256 64 56 512" "1024 256 14 512" "128 512 28 512"; do
    set -- $sh
    timeout -k 10 120 python3 bench/gemm_probe.py --op gemm --dtype f32 --C $1 --K $2 --H $3 --batch $4 --sweep $S | sed "s/^/$v /" >> $D/sweep.txt || exit 1
  done
done
python3 - <<PY
import json, collections
t = collections.defaultdict(dict)
for l in open("$D/sweep.txt"):
    v, js = l.split(" ", 1)
    d = json.loads(js)
    if "us" not in d: continue
    t[(d["C"], d["K"], d["H"], d["cfg"])][v] = d["us"]
for k in sorted(t):
    a = t[k]
    if "new" in a and "old" in a: print(k, "new %.1f old %.1f  %+.1f%%" % (a["new"], a["old"], 100 * (a["old"] / a["new"] - 1)))
PY
