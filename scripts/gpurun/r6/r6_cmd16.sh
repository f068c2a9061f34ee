#!/bin/bash
# r6c16: PMC counter passes over the fp32 / bf16x6 stem kernels (bench/stem_x6_probe.py, bs128)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6c16
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  PYTHONPATH=. timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --kernel-include-regex stem --output-format csv -d $OUT/stem_p$i -o run -- python3 bench/stem_x6_probe.py > $OUT/stem_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY' > $OUT/summary.txt
import collections, csv, glob
d = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob("gpurun_out/r6c16/stem_p*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    ids = collections.defaultdict(set)
    for r in rows:
        ids[r["Kernel_Name"]].add(r["Dispatch_Id"])
    for r in rows:
        d[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"]) / len(ids[r["Kernel_Name"]])
for k, c in d.items():
    if "SQ_INSTS_MFMA" not in c:
        continue
    w = max(c["SQ_WAVE_CYCLES"], 1.0)
    print(k[:90])
    print("   per dispatch: mfma %.0f valu %.0f lds %.0f salu %.0f | gui_active/8 %.0f | mfma_busy %.0f"
          " | wait_any %.1f%% wait_inst %.1f%% wait_lds %.1f%% | lds_conflict/active %.3f | vmem_cyc %.0f"
          % (c["SQ_INSTS_MFMA"], c["SQ_INSTS_VALU"], c["SQ_INSTS_LDS"], c["SQ_INSTS_SALU"], c["GRBM_GUI_ACTIVE"] / 8,
             c["SQ_VALU_MFMA_BUSY_CYCLES"], 100 * c["SQ_WAIT_ANY"] / w, 100 * c["SQ_WAIT_INST_ANY"] / w,
             100 * c["SQ_WAIT_INST_LDS"] / w, c["SQ_LDS_BANK_CONFLICT"] / max(1.0, c["SQ_LDS_IDX_ACTIVE"]),
             c["SQ_INST_CYCLES_VMEM"]))
PY
cat $OUT/summary.txt
find $OUT -name '*.csv' -size +4M -delete
