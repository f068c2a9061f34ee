#!/bin/bash
# r6c49: side-stream size gate at bs512: fork only grad-weights >= 25 / 60 GFLOP vs >= 8 (default: every
# ResNet-50 bs512 grad-weight); interleaved fp32 + bf16
set -u
D=gpurun_out/r6c49
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --ref-batch 0"
for r in 1 2; do
  GKSGD_WGRAD_STREAM_MIN_GFLOP=25 timeout -k 10 400 $B --json-out $D/g25_$r.json > $D/g25_$r.log 2>&1 || exit 1
  GKSGD_WGRAD_STREAM_MIN_GFLOP=60 timeout -k 10 400 $B --json-out $D/g60_$r.json > $D/g60_$r.log 2>&1 || exit 1
  timeout -k 10 400 $B --json-out $D/g8_$r.json > $D/g8_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("g25_1", "g60_1", "g8_1", "g25_2", "g60_2", "g8_2"):
    d = json.load(open("gpurun_out/r6c49/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
