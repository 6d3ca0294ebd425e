#!/usr/bin/env python3
"""Where does the skinny GEMM differ from torch: per mode, rel error and the pattern of
bad rows / columns (store epilogue, partials + splitk epilogue)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip import _ffi as ff
dev = torch.device("cuda:0")
for (M, N, K) in [(125, 2048, 6144), (16, 256, 512), (128, 64, 512), (1, 64, 128)]:
    g = torch.Generator(device=dev).manual_seed(1)
    A = torch.randn(M, K, device=dev, generator=g).bfloat16()
    W = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    ref = A.float() @ W.float().t()
    for mode in (102, 103, 104, 100):
        C = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
        rc = ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(C), N, M, N, K, None, 0, mode,
                                          ff.stream_ptr())
        torch.cuda.synchronize()
        err = (C.float() - ref).abs()
        bad = err > 0.05 * ref.abs().max()
        rows = bad.any(1).nonzero().flatten().tolist()
        cols = bad.any(0).nonzero().flatten().tolist()
        print(f"M={M} N={N} K={K} mode={mode} rc={rc} rel={float(err.norm()/ref.norm()):.4f} badrows={len(rows)} {rows[:8]} badcols={len(cols)} {cols[:8]}", flush=True)
        if bad.any() and M * N <= 16384:
            # does C match a shifted/partial product?
            for ks in range(0, K, 32):
                part = A[:, :ks].float() @ W[:, :ks].float().t()
                if float((C.float() - part).norm() / (part.norm() + 1e-9)) < 0.02:
                    print("   matches the product over K =", ks)
                    break
