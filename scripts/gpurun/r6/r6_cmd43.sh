#!/bin/bash
# r6c43: fp32 with only the Winograd grad-weights forked (GKSGD_WGRAD_STREAM_KINDS=wino: the x6 TN grad-weights,
# which stretch the critical-path GEMMs by sharing CUs, stay inline) vs every HIP grad-weight forked; interleaved
set -u
D=gpurun_out/r6c43
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --no-bf16-phase --ref-batch 0"
for r in 1 2; do
  GKSGD_WGRAD_STREAM_KINDS=wino timeout -k 10 400 $B --json-out $D/wino_$r.json > $D/wino_$r.log 2>&1 || exit 1
  timeout -k 10 400 $B --json-out $D/all_$r.json > $D/all_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("wino_1", "all_1", "wino_2", "all_2"):
    d = json.load(open("gpurun_out/r6c43/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
