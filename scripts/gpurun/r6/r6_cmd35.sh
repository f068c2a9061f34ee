#!/bin/bash
# r6c35: side stream restricted to a CU slice (GKSGD_WGRAD_STREAM_CUS=64 / 128 of 256, hipExtStreamCreateWithCUMask)
# so the grad-weights never hold the CUs the critical path needs, vs the unmasked side stream; interleaved, fp32 + bf16
set -u
D=gpurun_out/r6c35
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --ref-batch 0"
for r in 1 2; do
  GKSGD_WGRAD_STREAM_CUS=64 timeout -k 10 400 $B --json-out $D/cu64_$r.json > $D/cu64_$r.log 2>&1 || exit 1
  GKSGD_WGRAD_STREAM_CUS=128 timeout -k 10 400 $B --json-out $D/cu128_$r.json > $D/cu128_$r.log 2>&1 || exit 1
  timeout -k 10 400 $B --json-out $D/all_$r.json > $D/all_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("cu64_1", "cu128_1", "all_1", "cu64_2", "cu128_2", "all_2"):
    d = json.load(open("gpurun_out/r6c35/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
