#!/usr/bin/env python3
"""Run torch.matmul (hipBLASLt) on the DiT GEMM shapes, for a kernel trace that names
the library's winning kernels (tile / wave / stream-K configuration in the name)."""
import torch
dev = torch.device("cuda:0")
for (M, N, K) in [(6000, 12288, 2048), (6000, 2048, 6144), (6000, 4096, 2048), (6000, 2048, 2048), (3000, 2048, 2048)]:
    A = torch.randn(M, K, device=dev).bfloat16()
    W = torch.randn(N, K, device=dev).bfloat16()
    for _ in range(3):
        torch.matmul(A, W.t())
    torch.cuda.synchronize()
    print(M, N, K, flush=True)
