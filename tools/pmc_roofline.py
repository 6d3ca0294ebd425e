#!/usr/bin/env python3
"""Counter evidence for bench.py's roofline kernel (the SwiGLU gate/up GEMM) from three
SEPARATE rocprofv3 --pmc passes over the same driver (tools/prof_dit.py), each with
--kernel-trace only (MI355X_MICROARCH.md §HBM and 'DVFS give-back'):

  pass F  FETCH_SIZE                 → HBM read bytes  = FETCH_SIZE KB × 1024 × 2
                                       (gfx950: FETCH_SIZE counts half the bytes of a
                                       16 B/lane streaming read, buffer_load … lds included)
  pass W  WRITE_SIZE                 → HBM write bytes = WRITE_SIZE KB × 1024 (exact for
                                       16-B stores)
  pass S  SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE, SQ_BUSY_CYCLES
          → mfma_busy_frac = MFMA-busy cycles / (1024 SIMDs × GRBM_GUI_ACTIVE / 8)
          → clock_GHz = GRBM_GUI_ACTIVE / 8 / the dispatch's duration IN THE SAME PASS;
            the guide notes this quotient reads high on dispatches shorter than ≈0.3 ms,
            so a value above the 2.4 GHz maximum is withheld (null) with the raw quotient
            kept as clock_quotient_GHz.

A SwiGLU call = every EPI_SWIGLU (template epilogue 3) dispatch of one DiT layer: the
main-grid kernel plus, for a tail-split call, the tail grid (gemm.hip gemm_tail_split).
Per-call figures sum those dispatch kinds; only kinds launched once per layer of every
forward (the DiT's 24 × forwards) are counted, so an encoder SwiGLU of another M is not.

usage: pmc_roofline.py FETCH_DB WRITE_DB SQ_DB OUT_JSON --M 6000 --calls 24 [--box B] [--git G]
"""
import argparse
import json
import re
import sqlite3
from collections import defaultdict


def _product_hash():
    import os as _os
    import sys as _sys
    _sys.path.insert(0, _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "ace-step-1.5_amd"))
    from acehip.provenance import product_hash
    return product_hash()


def _short(name):
    name = name.replace("acehip::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*\)$", "", name)


# position of the EPI template argument per GEMM kernel (gemm.hip): gemm_pp_kernel<BM, EPI, DBG,
# SPL, SCH>, gemm_w4_kernel<BM, BN, EPI, ...>, gemm_kernel<BM, BN, WM, WN, STAGES, EPI>,
# gemm_sk_kernel<EPI>
# gemm_pp_split_kernel<EPI>: the tail-split main + tail grids in one launch (round 5)
EPI_POS = {"gemm_pp_kernel": 1, "gemm_w4_kernel": 2, "gemm_kernel": 5, "gemm_sk_kernel": 0, "gemm_pp_split_kernel": 0}


def _is_swiglu(short):
    m = re.match(r"(gemm_\w*kernel)<(.*)>$", short)
    if not m or m.group(1) not in EPI_POS:
        return False
    args = [x.strip() for x in m.group(2).split(",")]
    i = EPI_POS[m.group(1)]
    return i < len(args) and args[i] == "3"


def dispatches(db, counters):
    """{(kernel, grid): [ {counter: value, 'dur_s': s}, ... ]} per dispatch, this pass only."""
    cur = sqlite3.connect(db).cursor()
    rows = defaultdict(dict)
    q = ("select dispatch_id, kernel_name, grid_size, counter_name, value, start, end "
         "from counters_collection")
    for did, name, grid, ctr, v, s, e in cur.execute(q):
        if ctr not in counters:
            continue
        r = rows[did]
        r["key"] = (_short(name), int(grid))
        r[ctr] = r.get(ctr, 0.0) + float(v)
        if s is not None and e is not None:
            r["dur_s"] = (e - s) * 1e-9
    out = defaultdict(list)
    for r in rows.values():
        out[r.pop("key")].append(r)
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch_db")
    p.add_argument("write_db")
    p.add_argument("sq_db")
    p.add_argument("out_json")
    p.add_argument("--M", type=int, required=True)
    p.add_argument("--calls", type=int, required=True, help="SwiGLU calls of the DiT in the driver run")
    p.add_argument("--box", default=None)
    p.add_argument("--git", default=None)
    a = p.parse_args()

    F = dispatches(a.fetch_db, {"FETCH_SIZE"})
    W = dispatches(a.write_db, {"WRITE_SIZE"})
    S = dispatches(a.sq_db, {"SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES"})
    keys = sorted(k for k in F if _is_swiglu(k[0]) and len(F[k]) == a.calls and len(W.get(k, [])) == a.calls
                  and len(S.get(k, [])) == a.calls)
    if not keys:
        raise SystemExit("no EPI_SWIGLU dispatch kind with %d launches in all three passes: %s" % (
            a.calls, sorted((k, len(v)) for k, v in F.items() if _is_swiglu(k[0]))))

    def mean(lst, c):
        return sum(d[c] for d in lst) / len(lst)

    per_kind = {}
    fetch = write = mfma = gui = dur = 0.0
    for k in keys:
        f_b = 2 * mean(F[k], "FETCH_SIZE") * 1024
        w_b = mean(W[k], "WRITE_SIZE") * 1024
        g = mean(S[k], "GRBM_GUI_ACTIVE")
        mb = mean(S[k], "SQ_VALU_MFMA_BUSY_CYCLES")
        d = mean(S[k], "dur_s")
        per_kind[f"{k[0]} grid={k[1]}"] = {"fetch_bytes": round(f_b), "write_bytes": round(w_b),
                                           "avg_us_in_sq_pass": round(d * 1e6, 2),
                                           "mfma_busy_frac": round(mb * 8 / (1024 * g), 4) if g else None}
        fetch += f_b
        write += w_b
        mfma += mb
        gui += g
        dur += d
    clk = gui / 8 / dur / 1e9 if dur else None
    sw = {"M": a.M, "kernels": keys and [f"{k[0]} grid={k[1]}" for k in keys],
          "hbm_bytes_per_call": round(fetch + write), "fetch_bytes_per_call": round(fetch),
          "write_bytes_per_call": round(write),
          "avg_us": round(dur * 1e6, 2),
          "mfma_busy_frac": round(mfma * 8 / (1024 * gui), 4) if gui else None,
          "clock_quotient_GHz": round(clk, 3) if clk else None,
          "clock_GHz": round(clk, 3) if clk and clk <= 2.4 else None,
          "per_kind": per_kind}
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | SQ_VALU_MFMA_BUSY_CYCLES,GRBM_GUI_ACTIVE,"
                     "SQ_BUSY_CYCLES, each its own --kernel-trace pass over tools/prof_dit.py (--forwards from the --calls count: 24 SwiGLU calls per forward)",
           "box": a.box, "git_head": a.git, "product_hash": _product_hash(),
           "note": "separate counter passes (not the bench's timed run); profiled passes run at a lower "
                   "clock than un-profiled ones (guide 'DVFS give-back' (2)); clock_GHz is withheld when "
                   "the GRBM quotient exceeds 2.4 GHz (short-dispatch bias)",
           "gemm_swiglu": sw}
    json.dump(doc, open(a.out_json, "w"), indent=1)
    print(json.dumps(sw, indent=1))


if __name__ == "__main__":
    main()
