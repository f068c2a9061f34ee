#!/bin/bash
# r5c44: retune only the grad-input GEMMs with the BN-backward epilogue (dgrad_bn keys; x62 BNB no longer
# spills), then an interleaved same-call A/B of the headline against the committed choices
set -u
D=gpurun_out/r5c44
mkdir -p $D
export TMPDIR=/tmp
GKSGD_GEMM_RETUNE_ONLY=dgrad_bn GKSGD_GEMM_SAVE=$D/choices.json timeout -k 10 900 python3 bench.py --gpus 1 --steps 10 --warmup 3 --no-native-phase --no-bf16-phase --json-out $D/tune.json > $D/tune.log 2>&1
rc=$?; echo tune_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/tune.log; exit $rc; }
python3 - <<PY
import json
old = {tuple(k): v for k, v in json.load(open("tuning/gemm_choices.json"))}
new = {tuple(k): v for k, v in json.load(open("$D/choices.json"))}
for k in sorted(new, key=str):
    if k[0] == "dgrad_bn" and old.get(k) != new[k]: print(k, old.get(k), "->", new[k])
PY
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-native-phase --json-out $D/old$i.json > $D/old$i.log 2>&1 || exit 1
  GKSGD_GEMM_CACHE=$D/choices.json timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-native-phase --json-out $D/new$i.json > $D/new$i.log 2>&1 || exit 1
done
python3 -c "
import json
for n in ('old1','new1','old2','new2'):
    d=json.load(open('$D/%s.json'%n)); print(n, d['value'], d['ms_per_step'], d.get('bf16_value'), d.get('ref_bs32_value'))"
