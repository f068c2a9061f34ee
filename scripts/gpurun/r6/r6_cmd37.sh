#!/bin/bash
# r6c37: BN streaming-pass grid under the side stream (GKSGD_BN_BLOCKS=512 / 2048 vs the default 1024):
# fewer BN workgroups may leave room for the concurrently running grad-weights; interleaved, fp32 + bf16
set -u
D=gpurun_out/r6c37
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --ref-batch 0"
for r in 1 2; do
  GKSGD_BN_BLOCKS=512 timeout -k 10 400 $B --json-out $D/b512_$r.json > $D/b512_$r.log 2>&1 || exit 1
  GKSGD_BN_BLOCKS=2048 timeout -k 10 400 $B --json-out $D/b2048_$r.json > $D/b2048_$r.log 2>&1 || exit 1
  timeout -k 10 400 $B --json-out $D/b1024_$r.json > $D/b1024_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("b512_1", "b2048_1", "b1024_1", "b512_2", "b2048_2", "b1024_2"):
    d = json.load(open("gpurun_out/r6c37/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
