#!/bin/bash
# PMC counter passes over the Winograd kernels (bench/wino_probe.hip builds):
#   VARIANT (probe binary suffix), C (channels), OP (0 fwd, 2 wgrad)
set -u
export TMPDIR=/tmp
OUT=${CTR_OUT:-gpurun_out/wctr}
mkdir -p $OUT
V=${VARIANT:-base}; C=${C:-128}; OP=${OP:-0}
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/${V}_c${C}_op${OP}_p$i -o run -- ${PROBE_DIR:-./bench/bin}/wino_probe_$V 512 5 $V $C $OP > $OUT/${V}_c${C}_op${OP}_p$i.log 2>&1
  echo "pass $i rc=$?"
done
