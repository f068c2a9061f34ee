#!/usr/bin/env python3
"""Summarise scripts/gpurun/r3/r3_counters.sh output: one row per probe with wall time
(median kernel duration), MFMA busy share, instruction ratios and waits.

mfma% = SQ_VALU_MFMA_BUSY_CYCLES / (median wall x 2.1 GHz x 1024 SIMDs) (the
busy counter already weights each MFMA by its pass count, so fp32 and bf16
rows compare on one scale; 2.1 GHz as in profiles/r02_gemm_counters.txt)."""
import collections
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1]
print("%-26s %-46s %8s %6s %9s %9s %6s %6s" % ("probe", "kernel", "wall_us", "mfma%", "valu/mfma", "salu/mfma",
                                                "wait", "stall"))
for pdir in sorted(glob.glob(os.path.join(root, "*/"))):
    name = os.path.basename(pdir.rstrip("/"))
    vals = collections.defaultdict(float)
    walls = []
    kname = None
    for f in sorted(glob.glob(os.path.join(pdir, "p*/run_counter_collection.csv"))):
        rows = list(csv.DictReader(open(f)))
        kf = "gemm_tn" if "wgrad" in name else "gemm_nt"
        rows = [r for r in rows if kf in r["Kernel_Name"]]
        if not rows:
            continue
        kname = rows[0]["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").replace("gk::", "")
        per = collections.defaultdict(float)
        disp = set()
        for r in rows:
            per[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
        for k, v in per.items():
            vals[k] = v / len(disp)
    for f in sorted(glob.glob(os.path.join(pdir, "p*/run_kernel_trace.csv"))):
        for r in csv.DictReader(open(f)):
            if ("gemm_tn" if "wgrad" in name else "gemm_nt") in r["Kernel_Name"]:
                walls.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    if not walls or not vals:
        print("%-26s (no data)" % name)
        continue
    wall = statistics.median(walls)
    mfma = vals.get("SQ_INSTS_MFMA", 0) or 1
    busy = vals.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
    wc = vals.get("SQ_WAVE_CYCLES", 0) or 1
    print("%-26s %-46s %8.1f %5.1f%% %9.2f %9.2f %5.1f%% %5.1f%%" % (
        name, kname[:46], wall, 100 * busy / (wall * 1e-6 * 2.1e9 * 1024), vals.get("SQ_INSTS_VALU", 0) / mfma,
        vals.get("SQ_INSTS_SALU", 0) / mfma, 100 * vals.get("SQ_WAIT_ANY", 0) / wc,
        100 * vals.get("SQ_WAIT_INST_ANY", 0) / wc))
