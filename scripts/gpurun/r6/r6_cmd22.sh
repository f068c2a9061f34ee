#!/bin/bash
# r6c22: the deferred shortcut BN backward in the consumer BN linked apply pass (dual apply, dz read once):
# GPU tests, then an interleaved headline A/B (GKSGD_BN_DEFER_BWD=1 default vs 0)
set -u
D=gpurun_out/r6c22
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_bn_defer_gpu.py tests/test_bn_gpu.py tests/test_e2e_gpu.py tests/test_precision_e2e_gpu.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert" $D/tests.log | head -20; exit $rc; }
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --ref-batch 0"
for r in 1 2; do
  timeout -k 10 400 $B --json-out $D/defer_$r.json > $D/defer_$r.log 2>&1 || exit 1
  GKSGD_BN_DEFER_BWD=0 timeout -k 10 400 $B --json-out $D/base_$r.json > $D/base_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("defer_1", "base_1", "defer_2", "base_2"):
    d = json.load(open("gpurun_out/r6c22/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
