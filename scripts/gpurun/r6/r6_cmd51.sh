#!/bin/bash
# r6c51: forked TN grad-weights with auto splits launched as 1 / 0.5 rounds of the chip's block slots
# (GKSGD_WGRAD_SIDE_QROUNDS=4 / 2) instead of two rounds (default), leaving CUs to the critical path; the TN
# kernel tests first (negative splits = quarter rounds), then interleaved fp32 + bf16
set -u
D=gpurun_out/r6c51
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_conv1x1_gpu.py tests/test_e2e_gpu.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -2 $D/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $D/tests.log | head; exit $rc; }
GKSGD_WGRAD_SIDE_QROUNDS=2 timeout -k 10 600 python3 -u -m pytest tests/test_e2e_gpu.py -x -q --timeout 300 --timeout-method thread -k side_stream > $D/tests_q2.log 2>&1
rc=$?; tail -2 $D/tests_q2.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --ref-batch 0"
for r in 1 2; do
  GKSGD_WGRAD_SIDE_QROUNDS=4 timeout -k 10 400 $B --json-out $D/q4_$r.json > $D/q4_$r.log 2>&1 || exit 1
  GKSGD_WGRAD_SIDE_QROUNDS=2 timeout -k 10 400 $B --json-out $D/q2_$r.json > $D/q2_$r.log 2>&1 || exit 1
  timeout -k 10 400 $B --json-out $D/q8_$r.json > $D/q8_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("q4_1", "q2_1", "q8_1", "q4_2", "q2_2", "q8_2"):
    d = json.load(open("gpurun_out/r6c51/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
