#!/bin/bash
# r6c34: reference batch (bs32) HIP-graph replay with the grad-weights as parallel graph branches
# (GKSGD_WGRAD_STREAM_GRAPH=1, every grad-weight forked) vs the single-stream graph, interleaved
# (r5c8 measured the branches 2x slower with the record_stream side stream)
set -u
D=gpurun_out/r6c34
mkdir -p $D
export TMPDIR=/tmp
R="python3 bench.py --gpus 1 --steps 10 --warmup 5 --model-phases none --no-native-phase --no-bf16-phase"
for r in 1 2; do
  GKSGD_WGRAD_STREAM_GRAPH=1 GKSGD_WGRAD_STREAM_MIN_GFLOP=0 timeout -k 10 400 $R --json-out $D/branch_$r.json > $D/branch_$r.log 2>&1 || exit 1
  timeout -k 10 400 $R --json-out $D/single_$r.json > $D/single_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("branch_1", "single_1", "branch_2", "single_2"):
    d = json.load(open("gpurun_out/r6c34/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
