#!/bin/bash
# r6c32: the training step on a high-priority stream (GKSGD_MAIN_PRIO=1: critical path dispatched ahead of the
# side-stream grad-weights) vs the default (side stream at the main stream's priority), interleaved, fp32 + bf16
set -u
D=gpurun_out/r6c32
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --ref-batch 0"
for r in 1 2; do
  GKSGD_MAIN_PRIO=1 timeout -k 10 400 $B --json-out $D/prio_$r.json > $D/prio_$r.log 2>&1 || exit 1
  timeout -k 10 400 $B --json-out $D/base_$r.json > $D/base_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("prio_1", "base_1", "prio_2", "base_2"):
    d = json.load(open("gpurun_out/r6c32/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
# reference batch (bs32) in the trainer's default eager execution (no HIP graph): side stream vs inline
R="python3 bench.py --gpus 1 --steps 10 --warmup 5 --model-phases none --no-native-phase --no-bf16-phase --ref-graph off"
for r in 1 2; do
  timeout -k 10 400 $R --json-out $D/ref_side_$r.json > $D/ref_side_$r.log 2>&1 || exit 1
  GKSGD_WGRAD_STREAM=0 timeout -k 10 400 $R --json-out $D/ref_inline_$r.json > $D/ref_inline_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("ref_side_1", "ref_inline_1", "ref_side_2", "ref_inline_2"):
    d = json.load(open("gpurun_out/r6c32/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
