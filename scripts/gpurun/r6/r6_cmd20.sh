#!/bin/bash
# r6c20: fresh-container rebuild check (smoke + the driver's default bench), then a
# retuned fp32 headline-only run whose tuner log gives per-GEMM-key timings (roofline table)
set -u
D=gpurun_out/r6c20
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 $D/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $D/bench1.json > $D/bench1.log 2>&1
rc=$?; echo bench1_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/bench1.log; exit $rc; }
python3 -c "
import json;d=json.load(open('$D/bench1.json'));print({k:d[k] for k in d if k.endswith('value') or k.endswith('ms_per_step') or k.endswith('error') or k.endswith('ratio')})"
GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_DUMP=$D/retune_f32.json timeout -k 10 900 python3 bench.py --gpus 1 --steps 10 --warmup 3 \
  --model-phases none --no-native-phase --no-bf16-phase --ref-batch 0 --json-out $D/retune_f32_bench.json > $D/retune_f32.log 2>&1
rc=$?; echo retune_rc=$rc; [ $rc -eq 0 ] || { tail -20 $D/retune_f32.log; exit $rc; }
python3 scripts/gemm_eff.py $D/retune_f32.json --batch 512 > $D/eff_f32.txt; head -60 $D/eff_f32.txt
