#!/usr/bin/env python3
"""The counter evidence for bench.py's roofline kernel and the L2 hit-rate table, in one GPU call
(each counter set in its OWN rocprofv3 pass with --kernel-trace only; the profiler runs as a
child process, this script never touches the GPU):

  pass fetch  FETCH_SIZE
  pass write  WRITE_SIZE
  pass sq     SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
  pass tcc    TCC_HIT_sum TCC_MISS_sum

over tools/prof_dit.py --forwards 2 (48 SwiGLU calls at M = 6000).  Writes
gpurun_out/<tag>_pmc_roofline.json (tools/pmc_roofline.py: traffic, MFMA-busy, clock, product
hash) and gpurun_out/<tag>_pmc_tcc.json (per kernel: TCC hits, misses, hit rate = hits / (hits +
misses) — MI355X_MICROARCH.md §L2 — and the L2-miss bytes at 128 B per miss), then deletes the
trace databases (gpurun_out is merged back only up to 64 MiB).

With MODE "vae": only the FETCH_SIZE and WRITE_SIZE passes, over tools/prof_dit.py --forwards 0
--vae (one 240 s decode), summarised by tools/pmc_vae.py → gpurun_out/<tag>_pmc_vae_traffic.json.

usage: pmc_final.py TAG [vae]"""
import glob
import json
import os
import shutil
import socket
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE"),
          ("sq", "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"), ("tcc", "TCC_HIT_sum TCC_MISS_sum")]


def run_pass(tag, name, counters, driver=("--forwards", "2")):
    d = os.path.join(REPO, "gpurun_out", f"{tag}_pmc_{name}")
    shutil.rmtree(d, ignore_errors=True)
    cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", *counters.split(), "--kernel-trace", "-d", d, "-o",
           "run", "--", "python3", os.path.join(REPO, "tools", "prof_dit.py"), *driver]
    print("==", " ".join(cmd), flush=True)
    with open(d + ".log", "w") as log:
        rc = subprocess.run(cmd, stdout=log, stderr=subprocess.STDOUT, cwd=REPO).returncode
    if rc:
        print(f"pass {name} failed rc={rc} (see {d}.log)", flush=True)
        sys.exit(rc)
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if not dbs:
        print(f"pass {name}: no database under {d}", flush=True)
        sys.exit(3)
    return d, dbs[0]


def main_vae(tag):
    dirs, dbs = [], {}
    for name, ctrs in PASSES[:2]:
        d, db = run_pass(tag, "vae_" + name, ctrs, driver=("--forwards", "0", "--vae"))
        dirs.append(d)
        dbs[name] = db
    rc = subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_vae.py"), dbs["fetch"], dbs["write"],
                         os.path.join(REPO, "gpurun_out", f"{tag}_pmc_vae_traffic.json")]).returncode
    for d in dirs:
        shutil.rmtree(d, ignore_errors=True)
    sys.exit(rc)


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "pmc"
    if len(sys.argv) > 2 and sys.argv[2] == "vae":
        main_vae(tag)
    dirs, dbs = [], {}
    for name, ctrs in PASSES:
        d, db = run_pass(tag, name, ctrs)
        dirs.append(d)
        dbs[name] = db
    out = os.path.join(REPO, "gpurun_out", f"{tag}_pmc_roofline.json")
    rc = subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_roofline.py"), dbs["fetch"], dbs["write"],
                         dbs["sq"], out, "--M", "6000", "--calls", "48", "--box", socket.gethostname()]).returncode
    if rc:
        sys.exit(rc)
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from pmc_sq import per_kernel  # noqa: E402
    tcc = per_kernel(dbs["tcc"])
    table = {}
    for k, v in tcc.items():
        h, m = v.get("TCC_HIT_sum", 0.0), v.get("TCC_MISS_sum", 0.0)
        if h + m <= 0:
            continue
        table[k] = {"launches": v["launches"], "avg_us": round(v.get("avg_us", 0.0), 1), "tcc_hit": h, "tcc_miss": m,
                    "hit_rate": round(h / (h + m), 4), "miss_bytes_128B": m * 128}
    table = dict(sorted(table.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["launches"]))
    with open(os.path.join(REPO, "gpurun_out", f"{tag}_pmc_tcc.json"), "w") as f:
        json.dump({"box": socket.gethostname(), "note": "per-launch averages over tools/prof_dit.py --forwards 2; "
                   "hit_rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)", "kernels": table}, f, indent=1)
    for k, v in list(table.items())[:12]:
        print(k[:80], v["hit_rate"], v["avg_us"], flush=True)
    for d in dirs:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
