#!/usr/bin/env python3
"""HBM traffic of one 240 s Oobleck decode per kernel family, from two SEPARATE rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE, each with --kernel-trace only) over `tools/prof_dit.py --forwards 0
--vae`, against the algorithmic bytes of the same launches (every activation read once and every
output written once, weights once per launch).  gfx950 correction as in tools/pmc_roofline.py:
HBM read bytes = FETCH_SIZE KB × 1024 × 2, write bytes = WRITE_SIZE KB × 1024.

Algorithmic bytes follow the decode's launch structure (csrc/vae.hip acehip_vae_decode):
  conv1 (k7, 64 → C0, snaked output only), per block: ConvTranspose (raw + snaked outputs), three
  residual units — C = 128: ru8/ru7 (read x_s, x; write x (units 0, 1), out_s), C ≥ 256: the k7
  conv (read x_s, write y_s) + the k1 conv with the residual (read y_s, x; write x (units 0, 1),
  x_s) — and conv_out (read x_s, write 2 fp32 channels).

usage: pmc_vae.py FETCH_DB WRITE_DB OUT_JSON [--T 6000]"""
import argparse
import json
import os
import re
import sqlite3
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ace-step-1.5_amd")]
from acehip.config import VAEConfig  # noqa: E402


def family(name):
    name = name.replace("acehip::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"[<(].*$", "", name)


def per_family(db, counter):
    cur = sqlite3.connect(db).cursor()
    tot = defaultdict(float)
    n = defaultdict(set)
    for did, name, v in cur.execute("select dispatch_id, kernel_name, value from counters_collection "
                                    "where counter_name = ?", (counter,)):
        f = family(name)
        tot[f] += float(v)
        n[f].add(did)
    return tot, {k: len(v) for k, v in n.items()}


def algorithmic(T, snake_in=True, gemm_convs=True):
    """snake_in (ACEHIP_VAE_SNAKE_IN=1, the default since round 5): the C = 128 blocks keep no x_s
    tensor — their ConvTranspose writes raw x only and each residual unit reads x once and writes
    one output (raw x' for units 0, 1; the next block's snaked input for unit 2)."""
    c = VAEConfig()
    B = 2                                                 # bf16 bytes
    fam = defaultdict(float)
    blocks = c.decoder_block_channels()
    c0 = blocks[0][0]
    fam["conv7_kernel"] += T * c.decoder_input_channels * B + T * c0 * B + 7 * c.decoder_input_channels * c0 * B
    # gemm_convs (ACEHIP_CONV7=2, ACEHIP_CONVT=1, round 5): the ConvTransposes and the C ≥ 256 k7
    # convs run on gemm_pp_kernel (EPI_CONV)
    kt = "gemm_pp_kernel" if gemm_convs else "conv_gemm_kernel"
    k7 = "gemm_pp_kernel" if gemm_convs else "conv7_kernel"
    L = T
    for cin, cout, s in blocks:
        Lo = L * s
        sin = snake_in and cout == 128
        fam[kt] += L * cin * B + (1 if sin else 2) * Lo * cout * B + cin * cout * 2 * s * B
        L = Lo
        for u in range(3):
            keep = u < 2
            if cout == 128 and sin:
                fam["ru8_kernel"] += 2 * L * cout * B + 8 * cout * cout * B
            elif cout == 128:
                fam["ru8_kernel"] += (2 + (2 if keep else 1)) * L * cout * B + 8 * cout * cout * B
            else:
                fam[k7] += 2 * L * cout * B + 7 * cout * cout * B
                fam["convp_kernel"] += (2 + (2 if keep else 1)) * L * cout * B + cout * cout * B
    fam["conv_out_kernel"] += L * 128 * B + L * 2 * 4
    return fam


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch_db")
    p.add_argument("write_db")
    p.add_argument("out_json")
    p.add_argument("--T", type=int, default=6000)
    p.add_argument("--no-snake-in", action="store_true", help="model of ACEHIP_VAE_SNAKE_IN=0")
    p.add_argument("--no-gemm-convs", action="store_true", help="model of ACEHIP_CONV7=1 ACEHIP_CONVT=0")
    a = p.parse_args()
    F, nF = per_family(a.fetch_db, "FETCH_SIZE")
    W, nW = per_family(a.write_db, "WRITE_SIZE")
    alg = algorithmic(a.T, snake_in=not a.no_snake_in, gemm_convs=not a.no_gemm_convs)
    out = {"T": a.T, "note": __doc__.split("\n\n")[0], "families": {}}
    tot_m = tot_a = 0.0
    for f in sorted(alg):
        m = 2 * F.get(f, 0.0) * 1024 + W.get(f, 0.0) * 1024
        out["families"][f] = {"launches": nF.get(f, 0), "hbm_read_bytes": round(2 * F.get(f, 0.0) * 1024),
                              "hbm_write_bytes": round(W.get(f, 0.0) * 1024), "algorithmic_bytes": round(alg[f]),
                              "ratio": round(m / alg[f], 3) if alg[f] else None}
        tot_m += m
        tot_a += alg[f]
    out["total"] = {"measured_bytes": round(tot_m), "algorithmic_bytes": round(tot_a), "ratio": round(tot_m / tot_a, 3)}
    json.dump(out, open(a.out_json, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
