#!/bin/bash
# r5c40: retune with the pre-split-B bf16x6 candidates (cfg family 3); interleaved A/B against the committed choices
# + BERT fp32; then the driver command again on the fresh choices
set -u
D=gpurun_out/r5c40
mkdir -p $D
export TMPDIR=/tmp

GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_SAVE=$D/choices_r50.json timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $D/tune_r50.json > $D/tune_r50.log 2>&1
rc=$?; echo tune_r50_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/tune_r50.log; exit $rc; }
GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_SAVE=$D/choices_bert.json timeout -k 10 600 python3 bench.py --model bert --steps 10 --warmup 3 --no-bf16-phase --json-out $D/tune_bert.json > $D/tune_bert.log 2>&1
rc=$?; echo tune_bert_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/tune_bert.log; exit $rc; }
python3 - <<PY
import json
d = {}
for f in ("$D/choices_r50.json", "$D/choices_bert.json"):
    for k, v in json.load(open(f)): d.setdefault(tuple(k), v)
json.dump([[list(k), list(v)] for k, v in sorted(d.items(), key=str)], open("$D/choices.json", "w"), indent=0)
print("keys", len(d))
PY
GKSGD_GEMM_CACHE=$D/choices.json timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $D/bench.json > $D/bench.log 2>&1
rc=$?; echo bench_rc=$rc
GKSGD_GEMM_CACHE=$D/choices.json timeout -k 10 600 python3 bench.py --model bert --steps 10 --warmup 3 --no-bf16-phase --json-out $D/bert.json > $D/bert.log 2>&1
rc=$?; echo bert_rc=$rc
python3 -c "
import json
for n in ('tune_r50','bench','tune_bert','bert'):
    d=json.load(open('$D/%s.json'%n)); print(n, {k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step')})"
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-native-phase --json-out $D/old$i.json > $D/old$i.log 2>&1 || exit 1
  GKSGD_GEMM_CACHE=$D/choices.json timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-native-phase --json-out $D/new$i.json > $D/new$i.log 2>&1 || exit 1
done
python3 -c "
import json
for n in ('old1','new1','old2','new2'):
    d=json.load(open('$D/%s.json'%n)); print(n, d['value'], d['ms_per_step'], d.get('bf16_value'), d.get('ref_bs32_value'))"
