#!/bin/bash
# PMC counter passes over the fp32 stem kernels (scripts/stem_f32_probe.py)
set -u
export TMPDIR=/tmp
OUT=${CTR_OUT:-gpurun_out/sctr}
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/stem_p$i -o run -- python3 scripts/stem_f32_probe.py 512 3 both > $OUT/stem_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for k in stem_f32_fwd_kernel stem_f32_wgrad_kernel; do
  echo "== $k"; python3 scripts/wino_ctr_summary.py $OUT $k
done > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
find $OUT -name '*.csv' -size +4M -delete
