#!/bin/bash
# r6c8: HIP-graph replay of the LSTM step -- graph GPU tests (incl. the
# dist_trainer --hip-graph CLI), then the LSTM bench with its reference-batch
# phase replayed (default on one GPU) vs eager, and the bs128 phase graphed
set -u
D=gpurun_out/r6c8
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_graph_gpu.py -x -q --timeout 600 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --gpus 1 --model lstm --steps 20 --warmup 5 --model-phases none --no-native-phase --no-bf16-phase"
timeout -k 10 300 $B --json-out $D/lstm_graph.json > $D/lstm_graph.log 2>&1 || exit 1
timeout -k 10 300 $B --ref-graph off --json-out $D/lstm_eager.json > $D/lstm_eager.log 2>&1 || exit 1
timeout -k 10 300 $B --graph --ref-batch 0 --json-out $D/lstm_bs128_graph.json > $D/lstm_bs128_graph.log 2>&1 || exit 1
python3 - <<'PY'
import json
for f in ("lstm_graph", "lstm_eager", "lstm_bs128_graph"):
    d = json.load(open("gpurun_out/r6c8/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step") or k in ("final_loss", "graph_captures")})
PY
