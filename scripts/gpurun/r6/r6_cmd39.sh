#!/bin/bash
# r6c39: fp32 grad-weights as the fp32-MFMA form of their tuned bf16x6 tile (GKSGD_WGRAD_NATIVE=1: compute-bound
# on the matrix pipe, less operand traffic beside the memory-bound BN passes) on the side stream vs the default
set -u
D=gpurun_out/r6c39
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --no-bf16-phase --ref-batch 0"
for r in 1 2; do
  GKSGD_WGRAD_NATIVE=1 timeout -k 10 400 $B --json-out $D/native_$r.json > $D/native_$r.log 2>&1 || exit 1
  timeout -k 10 400 $B --json-out $D/x6_$r.json > $D/x6_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("native_1", "x6_1", "native_2", "x6_2"):
    d = json.load(open("gpurun_out/r6c39/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
