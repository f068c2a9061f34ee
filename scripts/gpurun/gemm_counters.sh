#!/bin/bash
# rocprofv3 counter passes over one hand-written kernel: bench/gemm_probe.py by
# default (PROBE=bench/stem_probe.py etc.), kernels whose name contains KFILTER.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${CTR_OUT:-gpurun_out/ctr}
mkdir -p $OUT
ARGS=${PROBE_ARGS:---op conv --cfg 124}
PROBE=${PROBE:-bench/gemm_probe.py}
export KFILTER=${KFILTER:-gemm_}
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  echo "=== pass $i: $set"
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $PROBE $ARGS > $OUT/p$i.log 2>&1
  echo "rc=$?"
  tail -2 $OUT/p$i.log
done
CTR_OUT=$OUT python3 - <<'PY'
import csv, collections, glob
import os
for f in sorted(glob.glob(os.environ.get("CTR_OUT", "gpurun_out/ctr") + "/p*/run_counter_collection.csv")):
    rows = [r for r in csv.DictReader(open(f)) if os.environ["KFILTER"] in r["Kernel_Name"]]
    if not rows:
        continue
    for kname in sorted(set(r["Kernel_Name"] for r in rows)):
      kr = [r for r in rows if r["Kernel_Name"] == kname]
      d = collections.defaultdict(float)
      for r in kr:
        d[r["Counter_Name"]] += float(r["Counter_Value"])
      nd = len(set(r["Dispatch_Id"] for r in kr))
      print(f, kname[:90])
      for k, v in sorted(d.items()):
        print("   %-28s %14.0f" % (k, v / nd))
PY
