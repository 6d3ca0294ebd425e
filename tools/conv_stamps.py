#!/usr/bin/env python3
"""Where a VAE conv GEMM tile's time goes (the C >= 256 decoder convs on the 256 x 256 ping-pong
tile, gemm.hip EPI_CONV): runs acehip_vae_conv at the 240 s decode's shapes on a GEMM_STAMPS build
(tools/ab_build.sh WT stamps -DGEMM_STAMPS) and prints, per launch round, the shader-clock cycles
of the prologue, the main loop and the epilogue (as tools/gemm_stamps.py), plus the launch time
and its TFLOP/s.  Only the first 16384 workgroups are stamped.

usage: conv_stamps.py [tools/ab/libacehip_stamps.so]   (SHAPES=k7_256,... to filter)"""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

LIB = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "tools", "ab", "libacehip_stamps.so")
lib = ctypes.CDLL(os.path.abspath(LIB))
P, I, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
lib.acehip_vae_conv.argtypes = [I, P, L, I, P, P, P, I, I, I, I, P, P, P, P, P]
lib.acehip_diag_gemm_stamps.argtypes = [P, I]
dev = torch.device("cuda:0")
# name: (kind, L_in, Cin, Cout, k, stride, dil, residual, snake out); the k = 7 convs write their
# Snake only (the decoder's form, which takes the implicit-GEMM path)
SHAPES = {"k7_256": (0, 1440000, 256, 256, 7, 1, 3, False, True),
          "k7_512": (0, 360000, 512, 512, 7, 1, 3, False, True),
          "k7_1024": (0, 60000, 1024, 1024, 7, 1, 3, False, True),
          "k1_256": (0, 1440000, 256, 256, 1, 1, 1, True, True),
          "convt_512_256": (1, 360000, 512, 256, 8, 4, 1, False, False),
          "convt_256_128": (1, 1440000, 256, 128, 8, 4, 1, False, False)}
if os.environ.get("SHAPES"):
    SHAPES = {k: v for k, v in SHAPES.items() if k in os.environ["SHAPES"].split(",")}
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
out = {}
for name, (kind, Lin, Cin, Cout, k, s, dil, has_res, snk) in SHAPES.items():
    g = torch.Generator(device=dev).manual_seed(0)
    Lout = Lin * s if kind == 1 else Lin
    x = (torch.rand(Lin, Cin, device=dev, generator=g) * 2 - 1).bfloat16()
    w = ((torch.rand(*((Cin, Cout, k) if kind == 1 else (Cout, Cin, k)), device=dev, generator=g) * 2 - 1)
         * 0.03).bfloat16()
    b = (torch.rand(Cout, device=dev, generator=g) * 0.1).bfloat16()
    res = (torch.rand(Lout, Cout, device=dev, generator=g) * 2 - 1).bfloat16() if has_res else None
    al = (torch.rand(Cout, device=dev, generator=g) * 0.2).bfloat16()
    be = (torch.rand(Cout, device=dev, generator=g) * 0.2).bfloat16()
    y = torch.empty(Lout, Cout, device=dev, dtype=torch.bfloat16)
    ys = torch.empty(Lout, Cout, device=dev, dtype=torch.bfloat16) if snk else None

    def call():
        assert lib.acehip_vae_conv(kind, x.data_ptr(), Lin, Cin, w.data_ptr(), b.data_ptr(),
                                   res.data_ptr() if res is not None else None, Cout, k, s, dil,
                                   None if (k == 7 and snk) else y.data_ptr(), al.data_ptr() if snk else None, be.data_ptr() if snk else None,
                                   ys.data_ptr() if snk else None, stream) == 0
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    assert lib.acehip_diag_gemm_stamps_clear() == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    call()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3
    taps = 2 if kind == 1 else k
    M = Lin + 1 if kind == 1 else Lin
    N = Cout * s if kind == 1 else Cout
    K = taps * Cin
    tiles = min(16384, ((M + 255) // 256) * (N // 256))
    buf = (ctypes.c_uint64 * (tiles * 2 * 8))()
    assert lib.acehip_diag_gemm_stamps(ctypes.cast(buf, P), tiles) == 0
    st = [[buf[(wg * 2) * 8 + i] for i in range(8)] for wg in range(tiles)]
    nz = sum(1 for r in st if any(r))
    st = [r for r in st if r[3] > r[0] > 0]
    if not st:
        print(name, "no stamped tiles", nz, "nonzero rows; sample", [buf[i] for i in range(16)], flush=True)
        continue
    r0 = min(r[4] for r in st)
    rows = sorted(({"start_us": (r[4] - r0) / 100.0, "end_us": (r[5] - r0) / 100.0, "pro": r[1] - r[0],
                    "main": r[2] - r[1], "epi": r[3] - r[2], "tot": r[3] - r[0]} for r in st),
                  key=lambda r: r["start_us"])
    nk = K // 64
    res_ = {"launch_us": round(us, 1), "tflops": round(2.0 * M * N * K / us * 1e-6, 1), "M": M, "N": N, "K": K,
            "nk": nk, "stamped_tiles": len(rows), "ideal_cyc_per_ktile": 2048, "rounds": []}
    for rd in range(0, min(len(rows), 256 * 6), 256):
        rr = rows[rd:rd + 256]
        med = {q: statistics.median(r[q] for r in rr) for q in ("pro", "main", "epi", "tot", "start_us", "end_us")}
        res_["rounds"].append({"n": len(rr), "start_us_med": round(med["start_us"], 2),
                               "end_us_med": round(med["end_us"], 2), "pro_cyc": int(med["pro"]),
                               "main_cyc": int(med["main"]), "main_cyc_per_ktile": round(med["main"] / nk, 1),
                               "mfma_frac_main": round(2048 * nk / med["main"], 3), "epi_cyc": int(med["epi"]),
                               "tot_cyc": int(med["tot"])})
    out[name] = res_
    print(name, json.dumps(res_), flush=True)
    del x, w, res, y, ys
    torch.cuda.empty_cache()
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(REPO, "gpurun_out", "conv_stamps.json"), "w"), indent=1)
