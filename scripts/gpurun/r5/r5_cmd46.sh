#!/bin/bash
# r5c46: selective retunes (fwd keys; dgrad keys) on the current kernels, each A/B'd against the committed
# choices in interleaved same-call runs of the driver's command
set -u
D=gpurun_out/r5c46
mkdir -p $D
export TMPDIR=/tmp
for dir in fwd dgrad; do
  GKSGD_GEMM_RETUNE_ONLY=$dir GKSGD_GEMM_SAVE=$D/choices_$dir.json timeout -k 10 900 python3 bench.py --gpus 1 --steps 5 --warmup 3 --no-native-phase --json-out $D/tune_$dir.json > $D/tune_$dir.log 2>&1
  rc=$?; echo tune_${dir}_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/tune_$dir.log; exit $rc; }
done
python3 - <<PY
import json
old = [[k, v] for k, v in json.load(open("tuning/gemm_choices.json"))]
for dir in ("fwd", "dgrad"):
    new = {tuple(k): v for k, v in json.load(open("$D/choices_%s.json" % dir))}
    out, n = [], 0
    for k, v in old:
        kt = tuple(k)
        if kt[0] == dir and kt in new and new[kt] != v:
            v = new[kt]; n += 1
        out.append([k, v])
    json.dump(out, open("$D/merged_%s.json" % dir, "w"), indent=0)
    print(dir, "changed", n)
PY
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-native-phase --json-out $D/old$i.json > $D/old$i.log 2>&1 || exit 1
  GKSGD_GEMM_CACHE=$D/merged_fwd.json timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-native-phase --json-out $D/fwd$i.json > $D/fwd$i.log 2>&1 || exit 1
  GKSGD_GEMM_CACHE=$D/merged_dgrad.json timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-native-phase --json-out $D/dgrad$i.json > $D/dgrad$i.log 2>&1 || exit 1
done
python3 -c "
import json
for n in ('old1','fwd1','dgrad1','old2','fwd2','dgrad2'):
    d=json.load(open('$D/%s.json'%n)); print(n, d['value'], d['ms_per_step'], d.get('bf16_value'), d.get('ref_bs32_value'))"
