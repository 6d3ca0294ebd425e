#!/usr/bin/env python3
"""Run one GEMM variant on one DiT shape a few times (for rocprofv3 counter passes).
usage: gemm_one.py <variant> <shape: down|qkv|o|swiglu> [reps]"""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip import _ffi as ff  # noqa: E402

SH = {"down": (6000, 2048, 6144, 0), "qkv": (6000, 4096, 2048, 0), "o": (6000, 2048, 2048, 0),
      "swiglu": (6000, 12288, 2048, 3)}
v, name = int(sys.argv[1]), sys.argv[2]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
M, N, K, epi = SH[name]
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
W = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).bfloat16()
ldc = N // 2 if epi == 3 else N
C = torch.empty(M, ldc, device=dev, dtype=torch.bfloat16)
for _ in range(reps):
    ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(C), ldc, M, N, K, None, epi, v,
                                          ff.stream_ptr()))
torch.cuda.synchronize()
print("ok", v, name)
