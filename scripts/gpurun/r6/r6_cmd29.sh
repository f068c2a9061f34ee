#!/bin/bash
# r6c29: (1) why the grad-weight side stream is 4.6x slower in fp32 (r6c28: 492 vs 107 ms/step) while
# +5% in bf16: caching-allocator counters per step (bench/stream_probe.py), fp32 side / inline, bf16 side;
# (2) BERT phase 71.5 ms in r6c27's default bench vs 67.4 in r6c6: standalone BERT vs the vocabulary-head
# A/B (GKSGD_LINEAR_PAD=0)
set -u
D=gpurun_out/r6c29
mkdir -p $D
export TMPDIR=/tmp
P="python3 bench/stream_probe.py --gpus 1 --steps 4 --warmup 3 --model-phases none --no-native-phase --ref-batch 0"
GKSGD_WGRAD_STREAM=1 timeout -k 10 300 $P > $D/probe_f32_side.log 2>&1; echo probe_f32_side_rc=$?; grep "^step" $D/probe_f32_side.log
timeout -k 10 300 $P > $D/probe_f32_inline.log 2>&1 || exit 1; grep "^step" $D/probe_f32_inline.log
GKSGD_WGRAD_STREAM=1 timeout -k 10 300 $P --amp bf16 > $D/probe_bf16_side.log 2>&1 || exit 1; grep "^step" $D/probe_bf16_side.log
timeout -k 10 300 $P --amp bf16 > $D/probe_bf16_inline.log 2>&1 || exit 1; grep "^step" $D/probe_bf16_inline.log
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --model bert"
timeout -k 10 400 $B --json-out $D/bert_1.json > $D/bert_1.log 2>&1 || exit 1
GKSGD_LINEAR_PAD=0 timeout -k 10 400 $B --json-out $D/bert_nopad.json > $D/bert_nopad.log 2>&1 || exit 1
timeout -k 10 400 $B --json-out $D/bert_2.json > $D/bert_2.log 2>&1 || exit 1
python3 - <<'PY'
import json
for f in ("bert_1", "bert_nopad", "bert_2"):
    d = json.load(open("gpurun_out/r6c29/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
