#!/bin/bash
# r6c4: bf16x6 LSTM step GEMM -- GPU tests, the step-GEMM probe (us + error vs
# fp64 per S), then the LSTM bench (bs128 + the reference's bs20) x6 vs the
# round-5 path (GKSGD_LSTM_X6=0)
set -u
D=gpurun_out/r6c4
mkdir -p $D
export TMPDIR=/tmp
echo skip-tests; rc=0

PYTHONPATH=. timeout -k 10 300 python3 bench/lstm_x6_probe.py > $D/probe.json 2> $D/probe.err
rc=$?; echo probe_rc=$rc; [ $rc -eq 0 ] || { tail -5 $D/probe.err; exit $rc; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r6c4/probe.json"))
for k in sorted(d):
    print(k, d[k])
PY
B="python3 bench.py --gpus 1 --model lstm --steps 20 --warmup 5 --model-phases none --no-native-phase --no-bf16-phase"
timeout -k 10 300 $B --json-out $D/lstm_x6.json > $D/lstm_x6.log 2>&1 || exit 1
GKSGD_LSTM_X6=0 timeout -k 10 300 $B --json-out $D/lstm_r5.json > $D/lstm_r5.log 2>&1 || exit 1
timeout -k 10 300 $B --json-out $D/lstm_x6b.json > $D/lstm_x6b.log 2>&1 || exit 1
python3 - <<'PY'
import json
for f in ("lstm_x6", "lstm_r5", "lstm_x6b"):
    d = json.load(open("gpurun_out/r6c4/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step") or k in ("final_loss",)})
PY
