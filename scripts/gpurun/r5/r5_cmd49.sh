#!/bin/bash
# r5c49: x62 A-fragment prefetch on every tile but 4x1, column statistics via LDS slots (no persistent
# stats / bias registers): GPU tests, per-cfg sweep and driver-command / BERT A/B vs variants/old (= HEAD)
set -u
D=gpurun_out/r5c49
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_x6_gpu.py > $D/t.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 $D/t.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
S=200001,200002,200003,200004,200006,200007
for v in new old; do
  if [ $v = old ]; then export GKSGD_EXT=variants/old/_C.so; else unset GKSGD_EXT; fi
  for sh in "768 3072 16 64" "3072 768 16 64" "768 2304 16 64" "768 768 16 64" "512 2048 7 512" "2048 512 7 512" "256 64 56 512" "1024 256 14 512"; do
    set -- $sh
    timeout -k 10 120 python3 bench/gemm_probe.py --op gemm --dtype f32 --C $1 --K $2 --H $3 --batch $4 --sweep $S | sed "s/^/$v /" >> $D/sweep.txt || exit 1
  done
  for sh in "128 28 128 1" "256 14 256 1" "256 56 512 2"; do
    set -- $sh
    timeout -k 10 120 python3 bench/gemm_probe.py --op conv --dtype f32 --C $1 --H $2 --K $3 --k 3 --stride $4 --batch 512 --sweep 200002,200003 | sed "s/^/$v /" >> $D/sweep.txt || exit 1
  done
  timeout -k 10 120 python3 bench/gemm_probe.py --op gemm_bnb --dtype f32 --C 512 --K 128 --H 28 --batch 512 --sweep 200002,200003 | sed "s/^/$v /" >> $D/sweep.txt || exit 1
done
unset GKSGD_EXT
python3 - <<PY
import json, collections
t = collections.defaultdict(dict)
for l in open("$D/sweep.txt"):
    v, js = l.split(" ", 1)
    d = json.loads(js)
    if "us" not in d: continue
    t[(d["op"], d["C"], d["K"], d["H"], d["cfg"])][v] = d["us"]
for k in sorted(t, key=str):
    a = t[k]
    if "new" in a and "old" in a: print(k, "new %.1f old %.1f  %+.1f%%" % (a["new"], a["old"], 100 * (a["old"] / a["new"] - 1)))
PY
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-native-phase --json-out $D/new$i.json > $D/new$i.log 2>&1 || exit 1
  GKSGD_EXT=variants/old/_C.so timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-native-phase --json-out $D/old$i.json > $D/old$i.log 2>&1 || exit 1
done
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --model bert --steps 10 --warmup 3 --no-bf16-phase --no-native-phase --json-out $D/bnew$i.json > $D/bnew$i.log 2>&1 || exit 1
  GKSGD_EXT=variants/old/_C.so timeout -k 10 600 python3 bench.py --model bert --steps 10 --warmup 3 --no-bf16-phase --no-native-phase --json-out $D/bold$i.json > $D/bold$i.log 2>&1 || exit 1
done
python3 -c "
import json
for n in ('new1','old1','new2','old2','bnew1','bold1','bnew2','bold2'):
    d=json.load(open('$D/%s.json'%n)); print(n, d['value'], d['ms_per_step'], d.get('bf16_value'), d.get('ref_bs32_value'))"
