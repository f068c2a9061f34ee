#!/bin/bash
# r6c17: parallel stem grad-weight reduce -- stem tests, probe (bs128 / bs512), headline A/B x6 stem vs GKSGD_STEM_X6=0
set -u
D=gpurun_out/r6c17
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_stem_gpu.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
PYTHONPATH=. timeout -k 10 120 python3 bench/stem_x6_probe.py > $D/probe128.json 2> $D/probe128.err || exit 1
PYTHONPATH=. N=512 timeout -k 10 120 python3 bench/stem_x6_probe.py > $D/probe512.json 2> $D/probe512.err || exit 1
cat $D/probe128.json $D/probe512.json
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --model-phases none --no-native-phase --no-bf16-phase"
for r in 1 2; do
  timeout -k 10 400 $B --json-out $D/x6_$r.json > $D/x6_$r.log 2>&1 || exit 1
  GKSGD_STEM_X6=0 timeout -k 10 400 $B --json-out $D/f32_$r.json > $D/f32_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("x6_1", "f32_1", "x6_2", "f32_2"):
    d = json.load(open("gpurun_out/r6c17/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
