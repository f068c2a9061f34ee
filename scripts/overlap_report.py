#!/usr/bin/env python3
"""Compute / communication-stream overlap from a rocprofv3 trace.

Input: the directory of ``rocprofv3 --marker-trace --kernel-trace`` CSVs of a
bench.py run with ``GKSGD_ROCTX=1``.  The comm-stream kernels (bucket
compression, exchange, decompress) are the ones on a different HIP stream
than the forward/backward kernels; this reports, per stream, the busy time
and how much of the side stream's kernel time ran while compute-stream
kernels were also executing, plus the host-side roctx phase ranges (gk/b<i>/
compress, gk/allgather/..., gk/update, gk/forward, gk/backward).

  python scripts/overlap_report.py gpurun_out/r2/marker [--out profiles/x.txt]
"""
import argparse
import collections
import csv
import os
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def overlap(a_iv, b_union):
    tot = 0
    j = 0
    for a, b in sorted(a_iv):
        while j < len(b_union) and b_union[j][1] <= a:
            j += 1
        k = j
        while k < len(b_union) and b_union[k][0] < b:
            tot += max(0, min(b, b_union[k][1]) - max(a, b_union[k][0]))
            k += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(os.path.join(a.dir, "run_kernel_trace.csv"))))
    by_stream = collections.defaultdict(list)
    names = collections.defaultdict(collections.Counter)
    for r in rows:
        s = (r["Queue_Id"], r.get("Stream_Id", "0"))
        iv = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        by_stream[s].append(iv)
        names[s][r["Kernel_Name"].split("(")[0][:60]] += 1
    busy = {s: sum(b - a for a, b in union(iv)) for s, iv in by_stream.items()}
    main_s = max(busy, key=busy.get)
    lines = ["# stream overlap from %s" % a.dir]
    mu = union(by_stream[main_s])
    for s, iv in sorted(by_stream.items(), key=lambda kv: -busy[kv[0]]):
        top = ", ".join("%s x%d" % (n, c) for n, c in names[s].most_common(4))
        if s == main_s:
            lines.append("compute stream queue=%s stream=%s: %d kernels, busy %.2f ms  [%s]" % (
                s[0], s[1], len(iv), busy[s] / 1e6, top))
        else:
            ov = overlap(iv, mu)
            ktime = sum(b - a for a, b in iv)
            lines.append("side stream queue=%s stream=%s: %d kernels, kernel time %.3f ms, of which %.3f ms "
                         "(%.0f%%) ran concurrently with compute-stream kernels  [%s]" % (
                             s[0], s[1], len(iv), ktime / 1e6, ov / 1e6, 100.0 * ov / max(ktime, 1), top))
    mpath = os.path.join(a.dir, "run_marker_api_trace.csv")
    if os.path.exists(mpath):
        ph = collections.defaultdict(list)
        for r in csv.DictReader(open(mpath)):
            ph[r["Function"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        lines.append("roctx host ranges (count, mean us):")
        for k in sorted(ph):
            v = ph[k]
            lines.append("  %-28s %4d  %9.1f" % (k, len(v), sum(v) / len(v)))
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
