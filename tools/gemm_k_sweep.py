#!/usr/bin/env python3
"""Per-tile fixed cost vs per-k-tile cost of the ping-pong GEMM: time at M=6000,
N=2048 (one round of 192x256 tiles) for growing K, plain store and residual epilogues."""
import os, sys, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip import _ffi as ff
dev = torch.device("cuda:0")
res = {}
for v, N in ((8, 2048), (7, 3072)):
    for K in (64, 256, 1024, 2048, 4096):
        M = 6000
        A = torch.randn(M, K, device=dev).bfloat16()
        W = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for epi in (0, 2):
            f = lambda: ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(C), N, M, N, K,
                                                              None, epi, v, ff.stream_ptr()))
            for _ in range(3): f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20): f()
            e1.record(); torch.cuda.synchronize()
            res[f"v{v} N{N} K{K} epi{epi}"] = round(e0.elapsed_time(e1) / 20 * 1e3, 1)
    print(json.dumps(res), flush=True)
