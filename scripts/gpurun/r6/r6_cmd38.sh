#!/bin/bash
# r6c38: LSTM reference batch (bs20) HIP graph with the three forked weight gradients (decoder, W_ih, W_hh of the
# last layer) as parallel graph branches beside the next layer's serial recurrence (GKSGD_WGRAD_STREAM_GRAPH=1)
# vs the single-stream graph, interleaved
set -u
D=gpurun_out/r6c38
mkdir -p $D
export TMPDIR=/tmp
M="python3 bench.py --gpus 1 --steps 20 --warmup 5 --model lstm --model-phases none --no-native-phase --no-bf16-phase"
for r in 1 2; do
  GKSGD_WGRAD_STREAM_GRAPH=1 timeout -k 10 400 $M --json-out $D/branch_$r.json > $D/branch_$r.log 2>&1 || exit 1
  timeout -k 10 400 $M --json-out $D/single_$r.json > $D/single_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("branch_1", "single_1", "branch_2", "single_2"):
    d = json.load(open("gpurun_out/r6c38/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
