#!/bin/bash
# r5c10: bf16x6 GEMM: config sweep + PMC counters (native cfg 3 vs x6 cfg 100003) at the BERT ffn1 shape
set -u
D=gpurun_out/r5c10
mkdir -p $D
export TMPDIR=/tmp
P="python3 bench/gemm_probe.py --op gemm --dtype f32 --C 768 --K 3072 --H 16 --batch 64"
S=1,2,3,4,11,12,13,14,101,102,103,104,201,202,203,204,1001,1002,1005,1006
X=$(echo $S | tr ',' '\n' | awk '{printf "%d,", $1+100000}')
timeout -k 10 120 $P --sweep $S$X > $D/sweep_bert.jsonl 2>&1 || exit 1
timeout -k 10 120 python3 bench/gemm_probe.py --op gemm --dtype f32 --C 512 --K 2048 --H 7 --batch 512 --sweep $S$X > $D/sweep_r50.jsonl 2>&1 || exit 1
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" \
           "SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM TA_BUSY_avr TA_TA_BUSY_sum"; do
  i=$((i+1))
  for cfg in 3 100003; do
    timeout -s KILL 60 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $D/c${cfg}_p$i -o run -- python3 bench/gemm_probe.py --op gemm --dtype f32 --C 768 --K 3072 --H 16 --batch 64 --cfg $cfg --iters 5 > $D/c${cfg}_p$i.log 2>&1
    echo "cfg $cfg pass $i rc=$?"
  done
done
cat $D/sweep_bert.jsonl $D/sweep_r50.jsonl | cut -c1-300
