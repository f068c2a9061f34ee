#!/bin/bash
# r6c45: one zero-padded copy of the output gradient shared by the padded grad-input and grad-weight GEMMs
# (K / N not multiples of 64: the LSTM's 10k-word decoder, BERT's vocabulary head): linear / LSTM / BERT GPU
# tests, then LSTM / BERT interleaved vs GKSGD_LINEAR_PAD_SHARE=0
set -u
D=gpurun_out/r6c45
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_linear_gpu.py tests/test_lstm_gpu.py tests/test_e2e_gpu.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -3 $D/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $D/tests.log | head; exit $rc; }
M="python3 bench.py --gpus 1 --steps 20 --warmup 5 --model-phases none --no-native-phase --no-bf16-phase"
for m in lstm bert; do
  for r in 1 2; do
    timeout -k 10 400 $M --model $m --json-out $D/${m}_share_$r.json > $D/${m}_share_$r.log 2>&1 || exit 1
    GKSGD_LINEAR_PAD_SHARE=0 timeout -k 10 400 $M --model $m --json-out $D/${m}_noshare_$r.json > $D/${m}_noshare_$r.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import json
for m in ("lstm", "bert"):
    for f in ("share_1", "noshare_1", "share_2", "noshare_2"):
        d = json.load(open("gpurun_out/r6c45/%s_%s.json" % (m, f)))
        print(m, f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
