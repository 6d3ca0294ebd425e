#!/usr/bin/env python3
"""GPU idle time inside a song: runs `bench.py --steps 1 --warmup 1 --no-cpu-baseline` (or the
given bench arguments) under rocprofv3 --kernel-trace as a child process, then over the LAST
song's window — from its first `apg_phase_kernel` dispatch's predecessor DiT forward start to the
end of its `conv_out_kernel` — sums the kernel busy time (union of dispatch intervals) against
the wall time and lists the largest idle gaps with the kernels on either side.  The trace
database is deleted afterwards (gpurun_out is merged back only up to 64 MiB).

usage: trace_gaps.py TAG [bench args ...]"""
import glob
import os
import re
import shutil
import sqlite3
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(n):
    n = n.replace("acehip::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*\)$", "", n)[:70]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "gaps"
    bargs = sys.argv[2:] or ["--steps", "1", "--warmup", "1", "--no-cpu-baseline"]
    d = os.path.join(REPO, "gpurun_out", f"{tag}_trace")
    shutil.rmtree(d, ignore_errors=True)
    cmd = ["timeout", "-s", "KILL", "400", "rocprofv3", "--kernel-trace", "-d", d, "-o", "run", "--", "python3",
           os.path.join(REPO, "bench.py"), *bargs]
    with open(d + ".log", "w") as log:
        rc = subprocess.run(cmd, stdout=log, stderr=subprocess.STDOUT, cwd=REPO).returncode
    if rc:
        print("rocprofv3 run failed", rc)
        sys.exit(rc)
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    cur = sqlite3.connect(db).cursor()
    names = {r[0]: short(r[1]) for r in cur.execute("select id, display_name from kernel_symbols")}
    rows = sorted(cur.execute("select kernel_id, start, end from rocpd_kernel_dispatch"), key=lambda r: r[1])
    outs = [i for i, r in enumerate(rows) if names.get(r[0], "").startswith("conv_out_kernel")]
    if len(outs) < 2:
        print("fewer than two decodes in the trace")
        sys.exit(4)
    i1 = outs[-1]
    i0 = outs[-2] + 1                      # everything after the previous song's decode
    win = rows[i0:i1 + 1]
    t0, t1 = win[0][1], win[-1][2]
    busy, end, gaps = 0, t0, []
    for k, (kid, s, e) in enumerate(win):
        if s > end:
            gaps.append((s - end, names.get(win[k - 1][0], "?") if k else "-", names.get(kid, "?")))
        busy += max(0, e - max(s, end))
        end = max(end, e)
    wall = t1 - t0
    print(f"song window: {len(win)} dispatches, wall {wall / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, "
          f"idle {(wall - busy) / 1e6:.2f} ms ({(wall - busy) / wall * 100:.2f} %)")
    agg = {}
    for g, a, b in gaps:
        key = (a, b)
        n, tot = agg.get(key, (0, 0))
        agg[key] = (n + 1, tot + g)
    tot = {}
    for kid, s_, e_ in win:
        n, t = tot.get(names.get(kid, "?"), (0, 0))
        tot[names.get(kid, "?")] = (n + 1, t + (e_ - s_))
    print("kernel time inside the window (top 25):")
    for nm, (n, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"  {t / 1e6:8.3f} ms  {n:6d} x {t / n / 1e3:8.1f} us  {nm}")
    print("largest idle totals by (before → after):")
    for (a, b), (n, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:15]:
        print(f"  {tot / 1e3:9.1f} us over {n:5d} gaps  {a}  →  {b}")
    shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
