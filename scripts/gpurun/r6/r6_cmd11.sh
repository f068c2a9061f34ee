#!/bin/bash
# r6c11: BN streaming cache policy in the full step -- non-temporal loads+stores
# (default build) vs plain loads+stores (variants/bnplain) vs plain stores only
# (variants/bnstplain): fp32 headline + bf16 phase, interleaved twice
set -u
D=gpurun_out/r6c11
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --model-phases none --no-native-phase"
for r in 1 2; do
  timeout -k 10 400 $B --json-out $D/nt_$r.json > $D/nt_$r.log 2>&1 || exit 1
  GKSGD_EXT=variants/bnplain/_C.so timeout -k 10 400 $B --json-out $D/plain_$r.json > $D/plain_$r.log 2>&1 || exit 1
  GKSGD_EXT=variants/bnstplain/_C.so timeout -k 10 400 $B --json-out $D/stplain_$r.json > $D/stplain_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("nt_1", "plain_1", "stplain_1", "nt_2", "plain_2", "stplain_2"):
    d = json.load(open("gpurun_out/r6c11/%s.json" % f))
    print(f, {k: d[k] for k in ("value", "ms_per_step", "bf16_value", "bf16_ms_per_step", "ref_bs32_value") if k in d})
PY
