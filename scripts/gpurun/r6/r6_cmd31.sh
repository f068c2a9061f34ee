#!/bin/bash
# r6c31: grad-weight side stream with held operand references (no record_stream): GPU tests, then
# interleaved A/B of the ResNet-50 bs512 headline + bf16 phase: inline / side / side without Winograd;
# LSTM and BERT (linear / LSTM grad-weights forked too) side vs inline
set -u
D=gpurun_out/r6c31
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_e2e_gpu.py -x -q --timeout 300 --timeout-method thread -k "side_stream" > $D/tests.log 2>&1
rc=$?; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --ref-batch 0"
for r in 1 2; do
  timeout -k 10 400 $B --json-out $D/side_$r.json > $D/side_$r.log 2>&1 || exit 1
  GKSGD_WGRAD_STREAM=0 timeout -k 10 400 $B --json-out $D/inline_$r.json > $D/inline_$r.log 2>&1 || exit 1
  GKSGD_WGRAD_STREAM_WINO=0 timeout -k 10 400 $B --json-out $D/nowino_$r.json > $D/nowino_$r.log 2>&1 || exit 1
done
M="python3 bench.py --gpus 1 --steps 20 --warmup 5 --model-phases none --no-native-phase --no-bf16-phase"
for m in lstm bert; do
  for r in 1 2; do
    timeout -k 10 400 $M --model $m --json-out $D/${m}_side_$r.json > $D/${m}_side_$r.log 2>&1 || exit 1
    GKSGD_WGRAD_STREAM=0 timeout -k 10 400 $M --model $m --json-out $D/${m}_inline_$r.json > $D/${m}_inline_$r.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import json
for f in ("side_1", "inline_1", "nowino_1", "side_2", "inline_2", "nowino_2", "lstm_side_1", "lstm_inline_1",
          "lstm_side_2", "lstm_inline_2", "bert_side_1", "bert_inline_1", "bert_side_2", "bert_inline_2"):
    d = json.load(open("gpurun_out/r6c31/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
