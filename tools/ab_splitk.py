#!/usr/bin/env python3
"""In-process A/B of the split-K knobs (ACEHIP_SPLITK_STAGES, ACEHIP_SPLITK_FILL) on the
10 s turbo GEMM shapes (M = Bc·S = 125), cold weights, interleaved rounds."""
import os, statistics, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip import _ffi as ff

dev = torch.device("cuda:0")
M = int(os.environ.get("M", "125"))
shapes = {"swiglu": (12288, 2048, 3), "down": (2048, 6144, 0), "qkv": (4096, 2048, 0), "o": (2048, 2048, 0)}
modes = [m.split(":") for m in os.environ.get("MODES", "2:1,3:1,2:2,3:2,2:4").split(",")]
for name, (N, K, epi) in shapes.items():
    A = torch.randn(M, K, device=dev).bfloat16()
    Ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(max(2, int(600e6 // (N * K * 2))))]
    ncol = N // 2 if epi == 3 else N
    C = torch.empty(M, ncol, device=dev, dtype=torch.bfloat16)
    res = {tuple(m): [] for m in modes}
    outs = {}
    for rnd in range(6):
        for st, fill in modes:
            os.environ["ACEHIP_SPLITK_STAGES"], os.environ["ACEHIP_SPLITK_FILL"] = st, fill
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for i in range(20):
                ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(Ws[i % len(Ws)]), K, ff.ptr(C), ncol, M, N,
                                                      K, None, epi, -1, ff.stream_ptr()))
            e1.record()
            torch.cuda.synchronize()
            if rnd:
                res[(st, fill)].append(e0.elapsed_time(e1) / 20 * 1e3)
            outs[(st, fill)] = C.float().clone()
    byts = 2.0 * (M * K + N * K + M * ncol)
    base = outs[tuple(modes[0])]
    for m in modes:
        us = statistics.median(res[tuple(m)])
        rel = float((outs[tuple(m)] - base).norm() / base.norm())
        print(f"{name} stages={m[0]} fill={m[1]}: {us:.1f} us  {byts / us / 1e3:.0f} GB/s  rel {rel:.1e}", flush=True)
