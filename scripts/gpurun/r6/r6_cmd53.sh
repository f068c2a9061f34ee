#!/bin/bash
# r6c53: a forked convolution's bias gradient (column pass over dy) on the side stream with its grad-weight
# (default) vs on the main stream (GKSGD_WGRAD_STREAM_BIAS=0): side-stream GPU tests incl. VGG-16 (conv biases),
# then VGG-16 bs512 interleaved
set -u
D=gpurun_out/r6c53
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_e2e_gpu.py tests/test_conv1x1_gpu.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -2 $D/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $D/tests.log | head; exit $rc; }
M="python3 bench.py --gpus 1 --steps 20 --warmup 5 --model vgg16 --model-phases none --no-native-phase --no-bf16-phase"
for r in 1 2; do
  timeout -k 10 400 $M --json-out $D/bias_side_$r.json > $D/bias_side_$r.log 2>&1 || exit 1
  GKSGD_WGRAD_STREAM_BIAS=0 timeout -k 10 400 $M --json-out $D/bias_main_$r.json > $D/bias_main_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("bias_side_1", "bias_main_1", "bias_side_2", "bias_main_2"):
    d = json.load(open("gpurun_out/r6c53/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
