#!/bin/bash
# r6c41: BN finalize inside the apply launch (GKSGD_BN_FIN_FUSE=1) under the side stream: the separate 4-block
# finalize kernels on the critical path wait for CU slots held by the grad-weights (bn_bwd_finalize 0.35 -> 1.67 ms
# per step, r6c36); interleaved vs default, fp32 + bf16
set -u
D=gpurun_out/r6c41
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --ref-batch 0"
for r in 1 2; do
  GKSGD_BN_FIN_FUSE=1 timeout -k 10 400 $B --json-out $D/fin_$r.json > $D/fin_$r.log 2>&1 || exit 1
  timeout -k 10 400 $B --json-out $D/base_$r.json > $D/base_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("fin_1", "base_1", "fin_2", "base_2"):
    d = json.load(open("gpurun_out/r6c41/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
