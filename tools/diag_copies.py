#!/usr/bin/env python3
"""Where do the blit-kernel copies (__amd_rocclr_copyBuffer) of a kernel trace come from:
for each one, the kernel dispatched just before and just after it on the same queue,
aggregated, with the copy's average duration.   usage: diag_copies.py DB"""
import re
import sqlite3
import sys
from collections import Counter, defaultdict

cur = sqlite3.connect(sys.argv[1]).cursor()
rows = cur.execute("select name, start, end, queue_id, grid_x from kernels order by start").fetchall()


def short(n):
    n = n.replace("acehip::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*\)$", "", n)[:70]


ctx = Counter()
dur = defaultdict(list)
for i, (n, s, e, q, gx) in enumerate(rows):
    if "copyBuffer" not in n:
        continue
    prev = next((short(r[0]) for r in reversed(rows[:i]) if r[3] == q and "copyBuffer" not in r[0]), "-")
    nxt = next((short(r[0]) for r in rows[i + 1:] if r[3] == q and "copyBuffer" not in r[0]), "-")
    ctx[(prev, nxt, gx)] += 1
    dur[(prev, nxt, gx)].append((e - s) * 1e-3)
print("copies:", sum(ctx.values()), "of", len(rows), "dispatches")
for k, c in ctx.most_common(25):
    print(f"{c:6d}  {sum(dur[k]) / len(dur[k]):8.1f} us  grid={k[2]:<9} after {k[0]}  before {k[1]}")
try:
    mc = cur.execute("select count(*), sum(size), avg(duration) from memory_copies").fetchone()
    print("memory_copies (runtime):", mc)
except sqlite3.Error as ex:
    print("memory_copies:", ex)
