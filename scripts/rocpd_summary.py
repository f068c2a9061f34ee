#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace run (rocpd SQLite output, ROCm 7.2's
default) into a per-kernel / per-category CSV, optionally restricted to the
last N steps (steps are delimited by a marker kernel that runs once per step).

usage: python scripts/rocpd_summary.py RUN_results.db OUT.csv --steps 10 --title "..."
       [--marker fused_sgd]  (count only dispatches after the (total-steps)-th marker)
"""
import argparse
import collections
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import category  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("out")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--title", default="")
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--marker", default=None,
                    help="substring of a kernel launched once per step; only the last --steps steps are counted")
    ap.add_argument("--marker-per-step", type=int, default=1,
                    help="dispatches of the marker kernel per step (e.g. 12 for a per-layer BERT kernel)")
    ap.add_argument("--sequence", default=None,
                    help="also write the ordered dispatches of the LAST step (name, grid, us) to this CSV")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x, vgpr_count, accum_vgpr_count, "
                     "lds_size from kernels order by start").fetchall()
    if a.marker:
        marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
        nper = max(1, a.marker_per_step)
        marks = marks[nper - 1::nper]   # the last marker dispatch of every step
        if len(marks) > a.steps:
            rows = rows[marks[-a.steps - 1] + 1:]
    if a.sequence and a.marker:
        marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
        last = rows[marks[-2] + 1:marks[-1] + 1] if len(marks) >= 2 else rows
        with open(a.sequence, "w") as f:
            f.write("i,us,grid,wg,kernel\n")
            for i, (name, s, e, gx, gy, gz, wx, vg, ag, lds) in enumerate(last):
                short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                f.write('%d,%.1f,"%d,%d,%d",%d,"%s"\n' % (i, (e - s) / 1e3, gx // max(wx, 1), gy, gz, wx, short[:150]))
    per = collections.defaultdict(lambda: [0, 0.0, None])
    for name, s, e, gx, gy, gz, wx, vg, ag, lds in rows:
        p = per[name]
        p[0] += 1
        p[1] += (e - s)
        p[2] = (gx // max(wx, 1), gy, gz, wx, vg, ag, lds)
    tot = sum(p[1] for p in per.values())
    # concurrency (several streams, e.g. the grad-weight side stream): union of
    # the kernel intervals vs their sum, over the counted window
    busy, cur_s, cur_e = 0, None, None
    for r in sorted(rows, key=lambda r: r[1]):
        if cur_e is None or r[1] > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = r[1], r[2]
        else:
            cur_e = max(cur_e, r[2])
    if cur_e is not None:
        busy += cur_e - cur_s
    wall = (max(r[2] for r in rows) - min(r[1] for r in rows)) if rows else 0
    cats = collections.Counter()
    for n, p in per.items():
        cats[category(n)] += p[1]
    with open(a.out, "w") as f:
        f.write("# %s\n" % a.title)
        f.write("# total kernel time %.1f ms over %d steps = %.2f ms/step\n" % (tot / 1e6, a.steps, tot / 1e6 / a.steps))
        f.write("# GPU wall %.2f ms/step, busy (union of kernel intervals) %.2f ms/step, kernel time run "
                "concurrently with another kernel %.2f ms/step\n" % (wall / 1e6 / a.steps, busy / 1e6 / a.steps,
                                                                     (tot - busy) / 1e6 / a.steps))
        f.write("category,ms_per_step,pct\n")
        for k, v in cats.most_common():
            f.write("%s,%.3f,%.1f\n" % (k, v / 1e6 / a.steps, 100.0 * v / tot))
        f.write("\nkernel,calls_per_step,ms_per_step,pct,us_per_call,grid(blocks_x,y,z),wg,vgpr,agpr,lds\n")
        for n, p in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
            g = p[2]
            f.write('"%s",%.1f,%.3f,%.1f,%.1f,"%s",%d,%d,%d,%d\n' % (
                n[:160].replace('"', "'"), p[0] / a.steps, p[1] / 1e6 / a.steps, 100.0 * p[1] / tot,
                p[1] / 1e3 / max(p[0], 1), "%d,%d,%d" % g[:3], g[3], g[4], g[5], g[6]))
    print(open(a.out).read()[:6000])


if __name__ == "__main__":
    main()
