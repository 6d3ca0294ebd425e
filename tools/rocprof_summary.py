#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace database (rocpd sqlite) per kernel:
calls, total ms, average µs, share — the same table --stats prints."""
import sqlite3
import sys
from collections import defaultdict


def summarize(db_path, top=40):
    cur = sqlite3.connect(db_path).cursor()
    names = {r[0]: (r[2] or r[1]) for r in cur.execute(
        "select id, kernel_name, truncated_kernel_name from kernel_symbols")}
    agg = defaultdict(lambda: [0, 0.0])
    for kid, s, e in cur.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        a = agg[names.get(kid, str(kid))]
        a[0] += 1
        a[1] += (e - s) * 1e-6  # ns → ms
    total = sum(v[1] for v in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]
    lines = ["| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for k, (n, ms) in rows:
        lines.append(f"| `{k[:110]}` | {n} | {ms:.2f} | {ms / n * 1e3:.1f} | {100 * ms / total:.1f} |")
    lines.append(f"| **total** | {sum(v[0] for v in agg.values())} | {total:.2f} | | 100 |")
    return "\n".join(lines)


if __name__ == "__main__":
    print(summarize(sys.argv[1]))
