#!/bin/bash
# PMC passes (scripts/gpurun/gemm_counters.sh) over the production GEMM kernels of
# ResNet-50 / BERT: MFMA-busy, VALU / SALU / LDS instruction mix, bank conflicts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for spec in "conv3x3_fwd_c64:--op conv --cfg 124 --C 64 --H 56" "conv3x3_fwd_c256:--op conv --cfg 125 --C 256 --H 14" \
            "conv1x1_fwd_64to256:--op gemm --cfg 24 --C 64 --K 256 --H 56" "wgrad3x3_c256:--op wgrad3 --cfg 5 --C 256 --H 14" \
            "bert_ffn_wgrad:--op lwgrad --cfg 5 --C 768 --K 3072 --H 512 --batch 32"; do
  tag=${spec%%:*}; args=${spec#*:}
  CTR_OUT=gpurun_out/ctr_top/$tag PROBE_ARGS="$args" bash scripts/gpurun/gemm_counters.sh > gpurun_out/ctr_top/$tag.log 2>&1
  echo "== $tag ($args)"; grep -E "SQ_|gemm_" gpurun_out/ctr_top/$tag.log | grep -v "^===" | tail -n 18
done
