#!/usr/bin/env python3
"""Per-kernel SQ / GRBM counters from a rocprofv3 --pmc pass (rocpd sqlite):
MFMA-busy cycles, wave waits and the effective clock per kernel (template
instance + grid), averaged over launches.

usage: pmc_sq.py DB [OUT_JSON]
Derived (per launch): clock_GHz = GRBM_GUI_ACTIVE / duration (the GPU's busy
clock ticks over the kernel's wall time, /8 when the counter sums the 8 XCDs);
mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (256 CUs x 4 SIMDs x busy cycles)
in the counter's own units (calibrated against the known MFMA count of the
SwiGLU GEMM in DESIGN.md)."""
import json
import re
import sqlite3
import sys
from collections import defaultdict


def _short(name):
    name = name.replace("acehip::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*\)$", "", name)


def per_kernel(db):
    cur = sqlite3.connect(db).cursor()
    vals = defaultdict(lambda: defaultdict(list))
    for name, grid, ctr, v in cur.execute(
            "select kernel_name, grid_size, counter_name, value from counters_collection"):
        vals[(_short(name), int(grid))][ctr].append(float(v))
    dur = defaultdict(list)
    try:
        for name, grid, s, e in cur.execute(
                "select kernel_name, grid_size, start, end from kernels"):
            dur[(_short(name), int(grid))].append((e - s) * 1e-9)
    except sqlite3.Error:
        # newer rocpd schemas: the dispatch times ride on the counter rows (one per dispatch)
        seen = {}
        for did, name, grid, s, e in cur.execute(
                "select dispatch_id, kernel_name, grid_size, start, end from counters_collection"):
            if s is not None and e is not None:
                seen[did] = ((_short(name), int(grid)), (e - s) * 1e-9)
        for k, d in seen.values():
            dur[k].append(d)
    out = {}
    for k, cs in vals.items():
        row = {c: sum(v) / len(v) for c, v in cs.items()}
        row["launches"] = len(next(iter(cs.values())))
        if dur.get(k):
            d = sum(dur[k]) / len(dur[k])
            row["avg_us"] = d * 1e6
            if "GRBM_GUI_ACTIVE" in row and d > 0:
                row["gui_active_per_s_GHz"] = row["GRBM_GUI_ACTIVE"] / d / 1e9
        out[f"{k[0]} grid={k[1]}"] = row
    return out


if __name__ == "__main__":
    t = per_kernel(sys.argv[1])
    for k, v in sorted(t.items(), key=lambda kv: -kv[1].get("avg_us", 0) * kv[1]["launches"])[:25]:
        print(k[:90], {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items()})
    if len(sys.argv) > 2:
        json.dump(t, open(sys.argv[2], "w"), indent=1)
