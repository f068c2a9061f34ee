#!/bin/bash
# r6c30: the fp32 side-stream pathology is bench-only (r6c28 492 ms/step; stream_probe 101-102 ms vs 103 inline,
# r6c29): probe at the bench's step counts, bench at the probe's, and bench without the exposed-comm marks
set -u
D=gpurun_out/r6c30
mkdir -p $D
export TMPDIR=/tmp
export GKSGD_WGRAD_STREAM=1
P="python3 bench/stream_probe.py --gpus 1 --model-phases none --no-native-phase --ref-batch 0"
timeout -k 10 300 $P --steps 24 --warmup 4 > $D/probe_long.log 2>&1 || exit 1; grep "^step" $D/probe_long.log | tr '\n' ';'; echo
B="python3 bench.py --gpus 1 --model-phases none --no-native-phase --no-bf16-phase --ref-batch 0"
timeout -k 10 300 $B --steps 4 --warmup 3 --json-out $D/b_short.json > $D/b_short.log 2>&1 || exit 1
timeout -k 10 300 $B --steps 20 --warmup 8 --json-out $D/b_long.json > $D/b_long.log 2>&1 || exit 1
GKSGD_BENCH_NO_MARKS=1 timeout -k 10 300 $B --steps 20 --warmup 8 --json-out $D/b_nomarks.json > $D/b_nomarks.log 2>&1 || exit 1
python3 - <<'PY'
import json
for f in ("b_short", "b_long", "b_nomarks"):
    d = json.load(open("gpurun_out/r6c30/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
