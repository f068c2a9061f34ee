#!/usr/bin/env python3
"""Summarise scripts/gpurun/wino_counters.sh passes: MFMA utilisation, VALU/LDS per
MFMA, wait shares and LDS bank-conflict ratio per Winograd kernel.
usage: python scripts/wino_ctr_summary.py gpurun_out/<dir>/ctr [kernel-substring,...]
(any kernel using v_mfma_f32_16x16x4_f32 only: the stem_f32 kernels too)"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
keys = sys.argv[2].split(",") if len(sys.argv) > 2 else ["wino_f23", "wino_wgrad_kernel"]
groups = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "*_p[12]/run_counter_collection.csv"))):
    groups[os.path.basename(os.path.dirname(f))[:-3]].append(f)
for g, files in groups.items():
    d = collections.defaultdict(float)
    name = ""
    for f in files:
        rows = [r for r in csv.DictReader(open(f)) if any(k in r["Kernel_Name"] for k in keys)]
        if not rows:
            continue
        name = rows[0]["Kernel_Name"][:60]
        ids = set(r["Dispatch_Id"] for r in rows)
        for r in rows:
            d[r["Counter_Name"]] += float(r["Counter_Value"]) / len(ids)
    if "SQ_INSTS_MFMA" not in d or "GRBM_GUI_ACTIVE" not in d:
        continue
    cyc = d["GRBM_GUI_ACTIVE"] / 8.0          # summed over the 8 XCDs
    mfma = d["SQ_INSTS_MFMA"] * 32 / (cyc * 1024)   # 16x16x4 f32: 32 cycles per SIMD
    w = d["SQ_WAVE_CYCLES"]
    print("%-22s %s" % (g, name))
    print("   mfma_util %.1f%%  valu/mfma %.2f  lds/mfma %.2f  lds_conflict %.3f  wait_any %.1f%%  wait_inst %.1f%%" % (
        100 * mfma, d["SQ_INSTS_VALU"] / d["SQ_INSTS_MFMA"], d["SQ_INSTS_LDS"] / d["SQ_INSTS_MFMA"],
        d["SQ_LDS_BANK_CONFLICT"] / max(1.0, d["SQ_LDS_IDX_ACTIVE"]), 100 * d["SQ_WAIT_ANY"] / w,
        100 * d["SQ_WAIT_INST_ANY"] / w))
