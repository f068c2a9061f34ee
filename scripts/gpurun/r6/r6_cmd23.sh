#!/bin/bash
# r6c23: static issue priority for the second-dispatched half of the 2-waves-per-SIMD kernels
# (x62 GEMMs, Winograd; variants/prio build, -DGK_X62_PRIO=1 -DGK_WINO_PRIO=1) vs the default build,
# interleaved; then a retuned bf16 headline-only run whose tuner log gives per-GEMM-key timings
set -u
D=gpurun_out/r6c23
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --gpus 1 --steps 20 --warmup 8 --model-phases none --no-native-phase --ref-batch 0"
for r in 1 2; do
  GKSGD_EXT=variants/prio/_C.so timeout -k 10 400 $B --json-out $D/prio_$r.json > $D/prio_$r.log 2>&1 || exit 1
  timeout -k 10 400 $B --json-out $D/base_$r.json > $D/base_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ("prio_1", "base_1", "prio_2", "base_2"):
    d = json.load(open("gpurun_out/r6c23/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
PY
GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_DUMP=$D/retune_bf16.json timeout -k 10 900 python3 bench.py --gpus 1 --steps 10 --warmup 3 \
  --model-phases none --no-native-phase --ref-batch 0 --json-out $D/retune_bf16_bench.json > $D/retune_bf16.log 2>&1
rc=$?; echo retune_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/retune_bf16.log; exit $rc; }
python3 scripts/gemm_eff.py $D/retune_bf16.json --batch 512 --dtype bf16 > $D/eff_bf16.txt; head -70 $D/eff_bf16.txt
