#!/usr/bin/env python3
"""Summarise scripts/gpurun/ctr_top.sh counter passes into one table per kernel:
wall us (kernel trace), MFMA pipe utilisation (16x16x32 bf16 MFMAs x 16
cycles / (wall x 2.1 GHz x 1024 SIMDs)), VALU and SALU instructions per MFMA,
LDS bank-conflict cycles / LDS-active cycles, and the share of wave cycles
parked in s_waitcnt / barriers (SQ_WAIT_ANY) and issue-stalled (SQ_WAIT_INST_ANY).

    python scripts/ctr_summary.py gpurun_out/ctr_top [--out profiles/r02_gemm_counters.txt]
"""
import argparse
import collections
import csv
import glob
import os

CLOCK = 2.1e9   # effective MFMA-loop clock under load (MI355X_MICROARCH.md DVFS notes)
SIMDS = 1024


def kernel_counters(d):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    nd = collections.defaultdict(set)
    for f in sorted(glob.glob(os.path.join(d, "p*/run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "gk::" not in k:
                continue
            out[k][r["Counter_Name"]] += float(r["Counter_Value"])
            nd[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    res = {}
    for k, cs in out.items():
        res[k] = {c: v / max(1, len(nd[(k, c)])) for c, v in cs.items()}
    return res


def kernel_wall(d):
    walls = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "p*/run_kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            walls[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: sorted(v)[len(v) // 2] for k, v in walls.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    lines = ["# rocprofv3 --pmc passes (scripts/gpurun/ctr_top.sh -> scripts/gpurun/gemm_counters.sh), one probe kernel each",
             "# mfma%% = MFMA instrs x 16 cyc / (median wall x %.1f GHz x %d SIMDs); valu/mfma, salu/mfma: instruction "
             "ratios (VALU count includes the MFMAs); lds_conf = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; wait / stall = "
             "SQ_WAIT_ANY / SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES" % (CLOCK / 1e9, SIMDS),
             "%-22s %-44s %8s %6s %9s %9s %8s %6s %6s" % ("probe", "kernel", "wall_us", "mfma%", "valu/mfma",
                                                        "salu/mfma", "lds_conf", "wait", "stall")]
    for d in sorted(glob.glob(os.path.join(a.root, "*/"))):
        tag = os.path.basename(os.path.normpath(d))
        cs, walls = kernel_counters(d), kernel_wall(d)
        for k, c in cs.items():
            mf = c.get("SQ_INSTS_MFMA", 0.0)
            w = walls.get(k, 0.0)
            util = mf * 16 / (w * 1e-6 * CLOCK * SIMDS) if w and mf else 0.0
            wc = c.get("SQ_WAVE_CYCLES", 0.0)
            lines.append("%-22s %-44s %8.1f %5.1f%% %9.2f %9.2f %8.3f %5.1f%% %5.1f%%" % (
                tag, k.replace("(anonymous namespace)::", "")[:44], w, 100 * util,
                c.get("SQ_INSTS_VALU", 0.0) / mf if mf else 0.0, c.get("SQ_INSTS_SALU", 0.0) / mf if mf else 0.0,
                c.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, c.get("SQ_LDS_IDX_ACTIVE", 0.0)),
                100 * c.get("SQ_WAIT_ANY", 0.0) / wc if wc else 0.0,
                100 * c.get("SQ_WAIT_INST_ANY", 0.0) / wc if wc else 0.0))
    text = "\n".join(lines) + "\n"
    print(text, end="")
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
