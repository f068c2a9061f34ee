#!/bin/bash
# PMC counters of the production GEMM kernels (fp32 headline + bf16), two passes
# per probe (scripts/gpurun/gemm_counters.sh), summarised by scripts/ctr_table.py.
set -u
D=${CTR_D:-gpurun_out/r3ctr}/ctr
mkdir -p $D
probe() {
  local name=$1 kf=$2; shift 2
  CTR_OUT=$D/$name PROBE_ARGS="$* --iters 10" KFILTER=$kf bash scripts/gpurun/gemm_counters.sh > $D/$name.log 2>&1
  echo "$name rc=$?"
}
probe f32_conv3x3_fwd_c64 gemm_nt --op conv --dtype f32 --C 64 --H 56 --k 3 --cfg 104 --mb 512
probe f32_conv3x3_fwd_c256 gemm_nt --op conv --dtype f32 --C 256 --H 14 --k 3 --cfg 204
probe f32_conv1x1_fwd_64to256 gemm_nt --op gemm --dtype f32 --C 64 --K 256 --H 56 --cfg 103 --mb 512
probe f32_wgrad3x3_c256 gemm_tn --op cwgrad --dtype f32 --C 256 --H 14 --k 3 --cfg 9
probe f32_wgrad1x1_256to64 gemm_tn --op cwgrad --dtype f32 --C 256 --K 64 --H 56 --k 1 --cfg 16
probe bf16_conv3x3_fwd_c64 gemm_nt --op conv --C 64 --H 56 --k 3 --cfg 124 --mb 512
probe bf16_conv3x3_fwd_c256 gemm_nt --op conv --C 256 --H 14 --k 3 --cfg 125
probe bf16_conv1x1_fwd_64to256 gemm_nt --op gemm --C 64 --K 256 --H 56 --cfg 213
probe bf16_wgrad3x3_c256 gemm_tn --op cwgrad --C 256 --H 14 --k 3 --cfg 5
probe bf16_wgrad1x1_256to64 gemm_tn --op cwgrad --C 256 --K 64 --H 56 --k 1 --cfg 3 --splits 128
python3 scripts/ctr_table.py $D > $D/table.txt
cat $D/table.txt
