#!/bin/bash
# r6c5: LSTM step GEMM autotuned per (direction, dtype, batch) + the big
# GEMMs (x W_ih, dx, dW_ih / dW_hh, the 10k softmax) on the HIP kernels over
# zero-padded operands when faster -- GPU tests, then the LSTM bench
# (bs128 + the reference's bs20): new vs the round-5 path
set -u
D=gpurun_out/r6c5
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_lstm_gpu.py tests/test_linear_gpu.py -x -q --timeout 600 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --gpus 1 --model lstm --steps 20 --warmup 5 --model-phases none --no-native-phase --no-bf16-phase"
OLD="env GKSGD_LSTM_SPLITK=fwd:64,bwd:1073741824 GKSGD_LINEAR_PAD=0"
GKSGD_GEMM_DUMP=$D/choices_1.json timeout -k 10 300 $B --json-out $D/lstm_new_1.json > $D/lstm_new_1.log 2>&1 || exit 1
GKSGD_LSTM_SPLITK=fwd:64,bwd:1073741824 GKSGD_LINEAR_PAD=0 timeout -k 10 300 $B --json-out $D/lstm_old_1.json > $D/lstm_old_1.log 2>&1 || exit 1
GKSGD_LINEAR_PAD=0 timeout -k 10 300 $B --json-out $D/lstm_steponly.json > $D/lstm_steponly.log 2>&1 || exit 1
timeout -k 10 300 $B --json-out $D/lstm_new_2.json > $D/lstm_new_2.log 2>&1 || exit 1
python3 - <<'PY'
import json
for f in ("lstm_new_1", "lstm_old_1", "lstm_steponly", "lstm_new_2"):
    d = json.load(open("gpurun_out/r6c5/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step") or k == "final_loss"})
c = json.load(open("gpurun_out/r6c5/choices_1.json"))
for r in c:
    if r[0][0] in ("lstm_step",) or (r[0][0].startswith("lin") and r[0][-1] == "pad"):
        print(r[0], r[1], [x for x in r[2] if isinstance(x[1], float)][:3])
PY
