#!/usr/bin/env python3
"""Fused head-post GEMM epilogue vs plain-store GEMM at the DiT QKV / cross-Q shapes (one process)."""
import os, sys, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip import _ffi as ff

dev = torch.device("cuda:0")
B, S, K = 2, 3000, 2048
M = B * S
A = torch.randn(M, K, device=dev).bfloat16()
cos = torch.randn(S, 128, device=dev).bfloat16(); sin = torch.randn(S, 128, device=dev).bfloat16()
qw = torch.ones(128, device=dev).bfloat16()


def timeit(fn, n=30):
    for _ in range(3): fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1e3, 1)


res = {}
for name, (nq, nk, nv, rope) in {"qkv": (16, 8, 8, True), "qkv_norope": (16, 8, 8, False),
                                  "crossq": (16, 0, 0, False), "v_only": (0, 0, 32, False)}.items():
    N = (nq + nk + nv) * 128
    W = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
    q = torch.empty(B, max(nq, 1), S, 128, device=dev, dtype=torch.bfloat16)
    k = torch.empty(B, max(nk, 1), S, 128, device=dev, dtype=torch.bfloat16)
    v = torch.empty(B, max(nv, 1), S, 128, device=dev, dtype=torch.bfloat16)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    hp = lambda: ff.check(ff.lib().acehip_gemm_headpost_bf16(
        ff.ptr(A), K, ff.ptr(W), K, B, S, nq, nk, nv, ff.ptr(qw), ff.ptr(qw), ff.ptr(cos) if rope else None,
        ff.ptr(sin) if rope else None, 1e-6, ff.ptr(q), ff.ptr(k), ff.ptr(v), ff.stream_ptr()))
    st = lambda: ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(C), N, M, N, K, None,
                                                       0, 8, ff.stream_ptr()))
    res[name] = {"headpost_us": timeit(hp), "store_v8_us": timeit(st)}
    print(name, res[name], flush=True)
print(json.dumps(res))
