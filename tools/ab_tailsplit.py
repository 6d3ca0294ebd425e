#!/usr/bin/env python3
"""In-process A/B of the GEMM tail split (ACEHIP_GEMM_TAILSPLIT) on the SwiGLU shapes
(240 s: M = 6000; 600 s: M = 15000), cold weights, interleaved rounds."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip import _ffi as ff

dev = torch.device("cuda:0")
for M in (6000, 15000):
    N, K = 12288, 2048
    A = torch.randn(M, K, device=dev).bfloat16()
    Ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(12)]
    C = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
    modes = os.environ.get("MODES", "1,0").split(",")
    res = {m: [] for m in modes}
    for rnd in range(6):
        for mode in modes:
            os.environ["ACEHIP_GEMM_TAILSPLIT"] = mode
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for i in range(24):
                ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(Ws[i % 12]), K, ff.ptr(C), N // 2, M, N,
                                                      K, None, 3, -1, ff.stream_ptr()))
            e1.record()
            torch.cuda.synchronize()
            if rnd:
                res[mode].append(e0.elapsed_time(e1) / 24 * 1e3)
    fl = 2.0 * M * N * K
    for mode, v in res.items():
        us = sorted(v)[len(v) // 2]
        print(f"M={M} tailsplit={mode}: {us:.1f} us  {fl / us / 1e6:.0f} TF/s")
