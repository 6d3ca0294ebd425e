#!/usr/bin/env python3
"""torch.matmul (hipBLASLt) on the DiT projection shapes, for a kernel trace: which macro tile /
MFMA / split the vendor library picks (the yardstick of tools/bench_gemm.py)."""
import torch
dev = torch.device("cuda:0")
for M, N, K in [(6000, 2048, 6144), (6000, 4096, 2048), (6000, 2048, 2048), (3000, 2048, 2048), (6000, 12288, 2048)]:
    A = torch.randn(M, K, device=dev).bfloat16()
    W = torch.randn(N, K, device=dev).bfloat16()
    for _ in range(3):
        torch.matmul(A, W.t())
    torch.cuda.synchronize()
