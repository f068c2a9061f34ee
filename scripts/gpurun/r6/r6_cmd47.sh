#!/bin/bash
# r6c47: grad-weight forks round-robin over 2 side streams (GKSGD_WGRAD_STREAMS=2) vs 1 (default); interleaved
set -u
D=gpurun_out/r6c47
mkdir -p $D
export TMPDIR=/tmp
GKSGD_WGRAD_STREAMS=2 timeout -k 10 600 python3 -u -m pytest tests/test_e2e_gpu.py -x -q --timeout 300 --timeout-method thread -k "side_stream" > $D/tests2.log 2>&1
rc=$?; tail -2 $D/tests2.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --ref-batch 0"
for r in 1 2; do
  GKSGD_WGRAD_STREAMS=2 timeout -k 10 400 $B --json-out $D/two_$r.json > $D/two_$r.log 2>&1 || exit 1
  timeout -k 10 400 $B --json-out $D/one_$r.json > $D/one_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("two_1", "one_1", "two_2", "one_2"):
    d = json.load(open("gpurun_out/r6c47/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
