#!/usr/bin/env python3
"""Dispatch timeline of a rocprofv3 --kernel-trace database: every kernel in start order with
its duration and the idle gap before it, from the first kernel at or after a start marker
(the N-th dispatch whose name contains MARK), for `count` dispatches; plus a per-name summary
of that window.  usage: timeline.py results.db [--mark NAME] [--nth N] [--count C]"""
import argparse
import re
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--mark", default="")
ap.add_argument("--nth", type=int, default=1)
ap.add_argument("--count", type=int, default=800)
a = ap.parse_args()
cur = sqlite3.connect(a.db).cursor()
names = {r[0]: re.sub(r"\(.*\)$", "", r[1].replace("acehip::(anonymous namespace)::", "").replace("void ", ""))
         for r in cur.execute("select id, display_name from kernel_symbols")}
rows = sorted(cur.execute("select kernel_id, start, end, grid_size_x, grid_size_y from rocpd_kernel_dispatch"),
              key=lambda r: r[1])
i0, seen = 0, 0
if a.mark:
    for i, r in enumerate(rows):
        if a.mark in names.get(r[0], ""):
            seen += 1
            if seen == a.nth:
                i0 = i
                break
win = rows[i0:i0 + a.count]
t0 = win[0][1]
prev_end = win[0][1]
agg = defaultdict(lambda: [0, 0.0, 0.0])
for kid, s, e, gx, gy in win:
    n = names.get(kid, str(kid))[:70]
    gap = (s - prev_end) * 1e-3
    print(f"{(s - t0) * 1e-3:10.1f} us  dur {(e - s) * 1e-3:8.1f}  gap {gap:6.1f}  {n} grid={gx}x{gy}")
    k = f"{n} grid={gx}x{gy}"
    agg[k][0] += 1
    agg[k][1] += (e - s) * 1e-3
    agg[k][2] += max(gap, 0)
    prev_end = max(prev_end, e)
print(f"# window: {len(win)} dispatches, {(prev_end - t0) * 1e-3:.1f} us wall, "
      f"{sum(v[1] for v in agg.values()):.1f} us busy, {sum(v[2] for v in agg.values()):.1f} us gaps")
for k, (c, d, g) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"# {c:5d} x  {d:9.1f} us busy  {g:8.1f} us gaps before  {k}")
