#!/usr/bin/env python3
"""Where a ping-pong GEMM tile's time goes: runs the DiT shapes on a GEMM_STAMPS build
(tools/ab_build.sh WT stamps -DGEMM_STAMPS) and prints, per launch round of workgroups,
the shader-clock cycles of the prologue (entry → first MFMA phase), the main loop and the
epilogue, the effective clock (shader cycles / real time) and the start skew.

usage: gemm_stamps.py [tools/ab/libacehip_stamps.so]   (SHAPES=swiglu,down,... to filter)"""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402

LIB = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "tools", "ab", "libacehip_stamps.so")
lib = ctypes.CDLL(os.path.abspath(LIB))
P, I = ctypes.c_void_p, ctypes.c_int
lib.acehip_gemm_bf16_ex.argtypes = [P, I, P, I, P, I, I, I, I, P, I, I, P]
lib.acehip_diag_gemm_stamps.argtypes = [P, I]
dev = torch.device("cuda:0")
# name: (M, N, K, epi, variant, BM)
SHAPES = {"swiglu": (6000, 12288, 2048, 3, 7, 256), "down": (6000, 2048, 6144, 2, 8, 192),
          "qkv": (6000, 4096, 2048, 0, 8, 192), "o": (6000, 2048, 2048, 2, 8, 192),
          "down256": (6000, 2048, 6144, 2, 7, 256),
          "o_half": (3000, 2048, 2048, 2, 13, 192)}
# MFMA cycles per K-tile per SIMD when the loop is back-to-back (16 cycles per 16x16x32)
IDEAL = {13: (96 // 16) * (64 // 16) * 2 * 16}
if os.environ.get("SHAPES"):
    SHAPES = {k: v for k, v in SHAPES.items() if k in os.environ["SHAPES"].split(",")}
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


out = {}
for name, (M, N, K, epi, var, BM) in SHAPES.items():
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
    nrot = max(1, int(600e6 // (N * K * 2)))
    W0 = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).bfloat16()
    Ws = [W0] + [W0.clone() for _ in range(nrot - 1)]
    ldc = N // 2 if epi == 3 else N
    C = torch.randn(M, ldc, device=dev).bfloat16()
    tiles = ((M + BM - 1) // BM) * (N // (128 if var == 13 else 256))
    for i in range(nrot + 2):
        assert lib.acehip_gemm_bf16_ex(A.data_ptr(), K, Ws[i % nrot].data_ptr(), K, C.data_ptr(), ldc, M, N, K,
                                       None, epi, var, stream) == 0
    torch.cuda.synchronize()
    assert lib.acehip_diag_gemm_stamps_clear() == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    assert lib.acehip_gemm_bf16_ex(A.data_ptr(), K, Ws[(nrot + 2) % nrot].data_ptr(), K, C.data_ptr(), ldc, M, N, K,
                                   None, epi, var, stream) == 0
    e1.record()
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * (tiles * 2 * 8))()
    assert lib.acehip_diag_gemm_stamps(ctypes.cast(buf, P), tiles) == 0
    st = [[buf[(w * 2 + gp) * 8 + i] for i in range(8)] for w in range(tiles) for gp in range(2)]
    g0 = st[0::2]
    r0 = min(s[4] for s in g0)
    rows = []
    for s in g0:
        pro, main, epi_c, tot = s[1] - s[0], s[2] - s[1], s[3] - s[2], s[3] - s[0]
        real_us = (s[5] - s[4]) / 100.0
        rows.append({"start_us": (s[4] - r0) / 100.0, "end_us": (s[5] - r0) / 100.0, "pro": pro, "main": main,
                     "epi": epi_c, "tot": tot, "ghz": tot / (real_us * 1e3) if real_us > 0 else 0.0,
                     "xcc": s[6] & 0xffffffff})
    rows.sort(key=lambda r: r["start_us"])
    nk = K // 64
    ideal = IDEAL.get(var, 2 * (BM // 2 // 16) * 4 * 2 * 16)   # cycles per K-tile per SIMD at 16 cyc/MFMA
    res = {"kernel_us_events": round(e0.elapsed_time(e1) * 1e3, 1),
           "span_us_real": round(max(r["end_us"] for r in rows), 1), "tiles": tiles, "nk": nk,
           "ideal_cyc_per_ktile": ideal, "rounds": []}
    cus = 256
    for rd in range(0, len(rows), cus):
        rr = rows[rd:rd + cus]
        med = {k: statistics.median(r[k] for r in rr) for k in ("pro", "main", "epi", "tot", "ghz", "start_us", "end_us")}
        res["rounds"].append({
            "n": len(rr), "start_us_med": round(med["start_us"], 2), "start_us_p90": round(pct([r["start_us"] for r in rr], 0.9), 2),
            "end_us_med": round(med["end_us"], 2), "pro_cyc": int(med["pro"]), "main_cyc": int(med["main"]),
            "main_cyc_per_ktile": round(med["main"] / nk, 1), "mfma_frac_main": round(ideal * nk / med["main"], 3),
            "epi_cyc": int(med["epi"]), "epi_cyc_p90": int(pct([r["epi"] for r in rr], 0.9)),
            "tot_cyc": int(med["tot"]), "ghz": round(med["ghz"], 3)})
    out[name] = res
    print(name, json.dumps(res), flush=True)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(REPO, "gpurun_out", "gemm_stamps.json"), "w"), indent=1)
