#!/bin/bash
# r6c19: lazy BN-backward operand (GKSGD_BN_LAZY=1: dx formed inside the producer's grad-input /
# grad-weight GEMMs, tuner choosing per GEMM between the lazy kernel and materialise + plain)
# re-measured under the bf16x6 GEMM family (round 3 measured it on fp32-MFMA kernels only)
set -u
D=gpurun_out/r6c19
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --no-bf16-phase"
for r in 1 2; do
  GKSGD_BN_LAZY=1 GKSGD_GEMM_DUMP=$D/lazy_tune_$r.json timeout -k 10 600 $B --json-out $D/lazy_$r.json > $D/lazy_$r.log 2>&1 || exit 1
  timeout -k 10 400 $B --json-out $D/base_$r.json > $D/base_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("lazy_1", "base_1", "lazy_2", "base_2"):
    d = json.load(open("gpurun_out/r6c19/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
