#!/bin/bash
# r6c40: BERT fp32 and LSTM fp32 kernel profiles at HEAD (grad-weight side stream), with the compression
# share per step; BERT k_cap = k (default) vs 4k/3 interleaved (fallback frequency of the 14 buckets)
set -u
D=gpurun_out/r6c40
mkdir -p $D
export TMPDIR=/tmp
for m in bert lstm; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof_$m -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 5 --model $m --model-phases none --no-native-phase --no-bf16-phase --ref-batch 0 --json-out $D/$m.json > $D/prof_$m.log 2>&1
  rc=$?; echo prof_${m}_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/prof_$m.log; exit $rc; }
  mk=mc_stats; per=1; [ $m = bert ] && per=14
  python3 scripts/rocpd_summary.py --marker $mk --marker-per-step $per --steps 10 --title "$m fp32 (bench.py --model $m), grad-weight side stream (r6c40)" $(find $D/prof_$m -name '*.db' | head -1) $D/${m}_summary.csv > $D/sum_$m.log 2>&1; echo sum_rc=$?
  find $D/prof_$m -name '*.db' -delete
  head -14 $D/${m}_summary.csv | cut -c1-200
done
M="python3 bench.py --gpus 1 --steps 20 --warmup 5 --model bert --model-phases none --no-native-phase --no-bf16-phase"
for r in 1 2; do
  timeout -k 10 400 $M --k-cap-factor 1.3334 --json-out $D/bert_kc43_$r.json > $D/bert_kc43_$r.log 2>&1 || exit 1
  timeout -k 10 400 $M --json-out $D/bert_kc1_$r.json > $D/bert_kc1_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("bert_kc43_1", "bert_kc1_1", "bert_kc43_2", "bert_kc1_2"):
    d = json.load(open("gpurun_out/r6c40/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step") or k.endswith("over_k") or k.endswith("ratio")})
PY
