#!/bin/bash
# r6c25: where does the bf16x6 Winograd's time go: probe timings of the default build and of
# timing-only variants without the patch loads / the U LDS-DMA / both; then two PMC passes
set -u
D=gpurun_out/r6c25
mkdir -p $D
export TMPDIR=/tmp
for v in base wx6noload wx6nodma wx6none; do
  if [ $v = base ]; then E=""; else E="GKSGD_EXT=variants/$v/_C.so"; fi
  env $E timeout -k 10 200 python3 bench/wx6_probe.py --batch 512 > $D/probe_$v.log 2>&1 || { tail -5 $D/probe_$v.log; exit 1; }
  echo "== $v"; grep -v "^{" $D/probe_$v.log | grep -v amdgpu.ids
done
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "wino" --output-format csv -d $D/ctr_p$i -o run -- python3 bench/wx6_probe.py --batch 512 > $D/ctr_p$i.log 2>&1
  echo "pass $i rc=$?"
done
find $D -name "*counter_collection.csv" | head
