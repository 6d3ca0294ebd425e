#!/usr/bin/env python3
"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Corrections per MI355X_MICROARCH.md §HBM: counters are in KB; on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) streaming reads, so it
is doubled; WRITE_SIZE is exact for 16-B stores.  Kernels are keyed by
template instance + grid (each GEMM shape its own row).

usage: pmc_traffic.py FETCH_DB WRITE_DB [OUT_JSON [M]]
"""
import json
import re
import sqlite3
import sys
from collections import defaultdict


def _short(name):
    name = name.replace("acehip::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*\)$", "", name)


def per_kernel(db, counter):
    cur = sqlite3.connect(db).cursor()
    agg = defaultdict(list)
    q = "select kernel_name, grid_size, value from counters_collection where counter_name = ?"
    for name, grid, v in cur.execute(q, (counter,)):
        agg[(_short(name), int(grid))].append(float(v))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def traffic(fetch_db, write_db):
    f = per_kernel(fetch_db, "FETCH_SIZE")
    w = per_kernel(write_db, "WRITE_SIZE")
    out = {}
    for k in f:
        if k in w:
            out[f"{k[0]} grid={k[1]}"] = {"fetch_bytes": 2 * f[k] * 1024, "write_bytes": w[k] * 1024,
                                          "hbm_bytes": 2 * f[k] * 1024 + w[k] * 1024}
    return out


# SwiGLU GEMM of the 240 s bench workload: M = 6000, N = 12288 (gate+up), K = 2048
SWIGLU_KEY = "gemm_kernel<256, 128, 4, 2, 2, 3>"


if __name__ == "__main__":
    t = traffic(sys.argv[1], sys.argv[2])
    for k, v in sorted(t.items(), key=lambda kv: -kv[1]["hbm_bytes"])[:30]:
        print(f"{k[:100]:100s} {v['hbm_bytes'] / 1e6:10.2f} MB  (fetch {v['fetch_bytes'] / 1e6:.2f}, write {v['write_bytes'] / 1e6:.2f})")
    if len(sys.argv) > 3:
        sw = [v for k, v in t.items() if re.match(r"gemm(_pp)?_kernel<.*, 3> grid=", k)]
        doc = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-trace on tools/prof_dit.py "
                         "(separate passes; FETCH x2 gfx950 correction; KB -> bytes)",
               "kernels": t}
        M = int(sys.argv[4]) if len(sys.argv) > 4 else 6000   # Bc·S of the profiled run
        # one SwiGLU GEMM call = the 256² ping-pong grid over rows [0, M1) + the tail rows as
        # 128×128 tiles (gemm_tail_split, gemm.hip; 256 CUs, N = 12288 → 48 column tiles)
        M1 = (((M + 255) // 256 * 48) // 256 * 256 // 48) * 256
        keys = [f"gemm_pp_kernel<256, 3> grid={(M1 // 256) * 48 * 512}"]
        if M1 < M:
            keys.append(f"gemm_kernel<128, 128, 2, 2, 2, 3> grid={((M - M1 + 127) // 128) * 96 * 256}")
        if all(k in t for k in keys):
            doc["gemm_swiglu_hbm_bytes_per_launch"] = sum(t[k]["hbm_bytes"] for k in keys)
            doc["gemm_swiglu_kernels"] = keys
            doc["gemm_swiglu_M"] = M
        elif sw:
            doc["gemm_swiglu_hbm_bytes_per_launch"] = max(v["hbm_bytes"] for v in sw)
            doc["gemm_swiglu_M"] = M
        json.dump(doc, open(sys.argv[3], "w"), indent=1)
