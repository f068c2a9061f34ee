#!/bin/bash
# r6c28: grad-weight side stream (GKSGD_WGRAD_STREAM=1) re-measured on the round-6 kernels (x62 GEMMs at
# 2 waves per SIMD leave VGPR / wave room for a BN pass to co-reside) vs inline, interleaved, fp32 + bf16
set -u
D=gpurun_out/r6c28
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --ref-batch 0"
for r in 1 2; do
  GKSGD_WGRAD_STREAM=1 timeout -k 10 400 $B --json-out $D/side_$r.json > $D/side_$r.log 2>&1 || exit 1
  timeout -k 10 400 $B --json-out $D/base_$r.json > $D/base_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("side_1", "base_1", "side_2", "base_2"):
    d = json.load(open("gpurun_out/r6c28/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
