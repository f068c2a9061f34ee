#!/bin/bash
# r6c2: e2e precision tests (fixed bound) + the GPU test files after them;
# A/B: k_cap = 4k/3 vs k; bs32 BN finalize in-apply (GKSGD_BN_FIN_FUSE) vs
# launches; BERT exposed comm with the strict bucket launch order
set -u
D=gpurun_out/r6c2
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_precision_e2e_gpu.py tests/test_shadow_gpu.py tests/test_stem_gpu.py tests/test_weight_prep_gpu.py tests/test_winograd_gpu.py tests/test_xent_gpu.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --model-phases none --no-native-phase"
for i in 1 2; do
  timeout -k 10 300 $B --json-out $D/kcap_default_$i.json > $D/kcap_default_$i.log 2>&1 || exit 1
  timeout -k 10 300 $B --k-cap-factor 1.0 --json-out $D/kcap_1_$i.json > $D/kcap_1_$i.log 2>&1 || exit 1
done
GKSGD_BN_FIN_FUSE=1 timeout -k 10 300 $B --no-bf16-phase --json-out $D/finfuse1.json > $D/finfuse1.log 2>&1 || exit 1
timeout -k 10 300 $B --no-bf16-phase --json-out $D/finfuse0.json > $D/finfuse0.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --model bert --model-phases none --no-native-phase --no-bf16-phase --ref-batch 0 --json-out $D/bert.json > $D/bert.log 2>&1 || exit 1
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6c2/*.json")):
    d = json.load(open(f))
    keys = [k for k in d if k.endswith("value") or k.endswith("ms_per_step") or k in ("selected_over_k", "effective_compression_ratio", "exposed_comm_ms", "compress_sync_timeouts")]
    print(f.split("/")[-1], {k: d[k] for k in keys})
PY
