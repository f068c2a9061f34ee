#!/bin/bash
# r5c47: fwd + dgrad retuned choices combined (r5c46), plus a wgrad-only retune on top; interleaved A/B
set -u
D=gpurun_out/r5c47
mkdir -p $D
export TMPDIR=/tmp
GKSGD_GEMM_CACHE=tuning/gemm_choices_fd.json GKSGD_GEMM_RETUNE_ONLY=wgrad GKSGD_GEMM_SAVE=$D/choices_w.json timeout -k 10 900 python3 bench.py --gpus 1 --steps 5 --warmup 3 --no-native-phase --json-out $D/tune_w.json > $D/tune_w.log 2>&1
rc=$?; echo tune_w_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/tune_w.log; exit $rc; }
python3 - <<PY
import json
base = [[k, v] for k, v in json.load(open("tuning/gemm_choices_fd.json"))]
new = {tuple(k): v for k, v in json.load(open("$D/choices_w.json"))}
out, n = [], 0
for k, v in base:
    kt = tuple(k)
    if kt[0] == "wgrad" and kt in new and new[kt] != v:
        v = new[kt]; n += 1
    out.append([k, v])
json.dump(out, open("$D/merged_all.json", "w"), indent=0)
print("wgrad changed", n)
PY
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-native-phase --json-out $D/old$i.json > $D/old$i.log 2>&1 || exit 1
  GKSGD_GEMM_CACHE=tuning/gemm_choices_fd.json timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-native-phase --json-out $D/fd$i.json > $D/fd$i.log 2>&1 || exit 1
  GKSGD_GEMM_CACHE=$D/merged_all.json timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-native-phase --json-out $D/all$i.json > $D/all$i.log 2>&1 || exit 1
done
python3 -c "
import json
for n in ('old1','fd1','all1','old2','fd2','all2'):
    d=json.load(open('$D/%s.json'%n)); print(n, d['value'], d['ms_per_step'], d.get('bf16_value'), d.get('ref_bs32_value'))"
