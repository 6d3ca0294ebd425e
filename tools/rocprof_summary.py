#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace database (rocpd sqlite): per kernel
(template instance + launch grid, so each GEMM shape is its own row) the
calls, total ms, average µs and share — the table ``--stats`` prints.

usage: rocprof_summary.py results.db [--by-name]
"""
import os
import re
import sqlite3
import sys
from collections import defaultdict

NAMEW = int(os.environ.get("NAMEW", "120"))


def _short(name: str) -> str:
    name = name.replace("acehip::(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*\)$", "", name)
    return name


def summarize(db_path, top=45, by_name=False):
    cur = sqlite3.connect(db_path).cursor()
    names = {r[0]: _short(r[1]) for r in cur.execute("select id, display_name from kernel_symbols")}
    agg = defaultdict(lambda: [0, 0.0])
    q = "select kernel_id, start, end, grid_size_x, grid_size_y, grid_size_z from rocpd_kernel_dispatch"
    for kid, s, e, gx, gy, gz in cur.execute(q):
        key = names.get(kid, str(kid))
        if not by_name and ("gemm" in key or "attn" in key):
            key = f"{key} grid={gx}x{gy}x{gz}"
        a = agg[key]
        a[0] += 1
        a[1] += (e - s) * 1e-6  # ns → ms
    total = sum(v[1] for v in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]
    lines = ["| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for k, (n, ms) in rows:
        lines.append(f"| `{k[:NAMEW]}` | {n} | {ms:.2f} | {ms / n * 1e3:.1f} | {100 * ms / total:.1f} |")
    lines.append(f"| **total** | {sum(v[0] for v in agg.values())} | {total:.2f} | | 100 |")
    return "\n".join(lines)


if __name__ == "__main__":
    print(summarize(sys.argv[1], by_name="--by-name" in sys.argv))
