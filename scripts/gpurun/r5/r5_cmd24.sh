#!/bin/bash
# r5c24: kernel profiles of the retuned fp32 headline and BERT fp32; PMC counters of the x62 row GEMM (BERT ffn2 shape)
set -u
D=gpurun_out/r5c24
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $D/prof -o prof -- python3 bench.py --steps 10 --warmup 5 --no-bf16-phase --no-native-phase --ref-batch 0 > $D/prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker reduce_records_kernel --steps 10 $(find $D/prof -name '*.db' | head -1) $D/r50_summary.txt > $D/sum.log 2>&1; echo sum_rc=$?
head -12 $D/r50_summary.txt
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $D/bprof -o prof -- python3 bench.py --model bert --steps 10 --warmup 3 --no-bf16-phase --no-native-phase > $D/bprof.log 2>&1
rc=$?; echo bprof_rc=$rc; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py --marker add_ln_fwd --marker-per-step 24 --steps 10 $(find $D/bprof -name '*.db' | head -1) $D/bert_summary.txt > $D/bsum.log 2>&1; echo bsum_rc=$?
head -12 $D/bert_summary.txt
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" \
           "SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $D/ctr_p$i -o run -- python3 bench/gemm_probe.py --op gemm --dtype f32 --C 3072 --K 768 --H 16 --batch 64 --cfg 200002 --iters 5 > $D/ctr_p$i.log 2>&1
  echo "pass $i rc=$?"
done
