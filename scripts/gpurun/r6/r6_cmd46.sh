#!/bin/bash
# r6c46: grad-weight forked AFTER the grad-input is issued (GKSGD_WGRAD_AFTER_DGRAD=1: the critical-path GEMM is
# dispatched first and the grad-weight overlaps the BN passes after it) vs before (default); interleaved fp32 + bf16
set -u
D=gpurun_out/r6c46
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_e2e_gpu.py -x -q --timeout 300 --timeout-method thread -k "side_stream" > $D/tests.log 2>&1
rc=$?; tail -2 $D/tests.log; [ $rc -eq 0 ] || exit $rc
GKSGD_WGRAD_AFTER_DGRAD=1 timeout -k 10 600 python3 -u -m pytest tests/test_e2e_gpu.py -x -q --timeout 300 --timeout-method thread -k "side_stream" > $D/tests_after.log 2>&1
rc=$?; tail -2 $D/tests_after.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --ref-batch 0"
for r in 1 2; do
  GKSGD_WGRAD_AFTER_DGRAD=1 timeout -k 10 400 $B --json-out $D/after_$r.json > $D/after_$r.log 2>&1 || exit 1
  timeout -k 10 400 $B --json-out $D/before_$r.json > $D/before_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("after_1", "before_1", "after_2", "before_2"):
    d = json.load(open("gpurun_out/r6c46/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
