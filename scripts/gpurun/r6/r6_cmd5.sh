#!/bin/bash
# r6c5: LSTM step GEMM autotuned per (direction, dtype, batch) -- GPU tests,
# then the LSTM bench (bs128 + the reference's bs20) tuned vs the round-5 rule
set -u
D=gpurun_out/r6c5
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_lstm_gpu.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --gpus 1 --model lstm --steps 20 --warmup 5 --model-phases none --no-native-phase --no-bf16-phase"
for i in 1 2; do
  GKSGD_GEMM_DUMP=$D/choices_$i.json timeout -k 10 300 $B --json-out $D/lstm_tuned_$i.json > $D/lstm_tuned_$i.log 2>&1 || exit 1
  GKSGD_LSTM_SPLITK="fwd:64,bwd:1073741824" timeout -k 10 300 $B --json-out $D/lstm_rule_$i.json > $D/lstm_rule_$i.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("lstm_tuned_1", "lstm_rule_1", "lstm_tuned_2", "lstm_rule_2"):
    d = json.load(open("gpurun_out/r6c5/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
c = json.load(open("gpurun_out/r6c5/choices_1.json"))
print([r[:2] for r in c if r[0][0] == "lstm_step"])
PY
