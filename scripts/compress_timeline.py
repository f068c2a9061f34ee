#!/usr/bin/env python3
"""Per-kernel timeline of one compress() call from a rocprofv3 --kernel-trace
run (rocpd SQLite): the median gaussian call of bench/kernels.py --only round2.
usage: python scripts/compress_timeline.py RUN_results.db"""
import sqlite3, sys, re, statistics
db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
rows = db.execute("select %s, start, end from kernels order by start" % ("name")).fetchall()
def short(n):
    n = n.replace("gk::(anonymous namespace)::", "").replace("void ", ""); n = re.sub(r"\(.*", "", n)
    return n[:60]
# find calls: sequences starting at stats_kernel and ending at select_kernel
calls = []
cur = None
for name, s, e in rows:
    sn = short(name)
    if sn.startswith("stats_kernel"):
        cur = [(sn, s, e)]
    elif cur is not None:
        cur.append((sn, s, e))
        if sn.startswith("select"):
            calls.append(cur); cur = None
print("calls", len(calls))
# first 70 calls = gaussian (30 settle + timeit + 40), take calls 35..60
sel = calls[31:60]
spans = [c[-1][2] - c[0][1] for c in sel]
print("gaussian span median us %.1f" % (statistics.median(spans) / 1e3))
c = sel[len(sel) // 2]
t0 = c[0][1]; prev = t0
for sn, s, e in c:
    print("%-60s start %7.1f dur %6.1f gap %5.1f" % (sn, (s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3))
    prev = e
