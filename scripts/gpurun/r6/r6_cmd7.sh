#!/bin/bash
# r6c7: conv bias gradient via the column pass + BERT vocabulary projection on
# the tuned (padded) GEMMs -- GPU tests, then same-box A/Bs
set -u
D=gpurun_out/r6c7
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_conv1x1_gpu.py tests/test_linear_gpu.py tests/test_attention_f32_gpu.py tests/test_e2e_gpu.py tests/test_shadow_gpu.py -x -q --timeout 600 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --model-phases none --no-native-phase --no-bf16-phase"
GKSGD_GEMM_DUMP=$D/choices_bert.json timeout -k 10 300 $B --model bert --ref-batch 0 --json-out $D/bert_new.json > $D/bert_new.log 2>&1 || exit 1
GKSGD_LINEAR_PAD=0 timeout -k 10 300 $B --model bert --ref-batch 0 --json-out $D/bert_old.json > $D/bert_old.log 2>&1 || exit 1
timeout -k 10 300 $B --model vgg16 --json-out $D/vgg_new.json > $D/vgg_new.log 2>&1 || exit 1
GKSGD_CONV_BIAS_COLSUM=0 timeout -k 10 300 $B --model vgg16 --json-out $D/vgg_old.json > $D/vgg_old.log 2>&1 || exit 1
timeout -k 10 300 $B --model bert --ref-batch 0 --json-out $D/bert_new2.json > $D/bert_new2.log 2>&1 || exit 1
timeout -k 10 300 $B --model vgg16 --json-out $D/vgg_new2.json > $D/vgg_new2.log 2>&1 || exit 1
python3 - <<'PY'
import json
for f in ("bert_new", "bert_old", "bert_new2", "vgg_new", "vgg_old", "vgg_new2"):
    d = json.load(open("gpurun_out/r6c7/%s.json" % f))
    print(f, {k: d[k] for k in d if k.endswith("value") or k.endswith("ms_per_step")})
c = json.load(open("gpurun_out/r6c7/choices_bert.json"))
for r in c:
    if r[0][-1] == "pad":
        print(r[0], r[1], [x for x in r[2] if isinstance(x[1], float)][:3])
PY
