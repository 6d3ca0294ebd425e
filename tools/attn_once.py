#!/usr/bin/env python3
"""Run one attention shape N times (driver for rocprofv3 counter passes).
usage: attn_once.py full|band|cross1 [N]   (ACEHIP_ATTN_PW selects the kernel)"""
import math, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip import _ffi as ff  # noqa: E402
SHAPES = {"full": (2, 16, 8, 3000, 3000, -1), "band": (2, 16, 8, 3000, 3000, 128), "cross1": (1, 16, 8, 3000, 641, -1)}
B, H, KV, Sq, Sk, w = SHAPES[sys.argv[1]]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(B, H, Sq, 128, device=dev, generator=g).bfloat16()
k = torch.randn(B, KV, Sk, 128, device=dev, generator=g).bfloat16()
v = torch.randn(B, KV, Sk, 128, device=dev, generator=g).bfloat16()
o = torch.empty(B, Sq, H * 128, device=dev, dtype=torch.bfloat16)
for _ in range(n):
    ff.check(ff.lib().acehip_attention_bf16(ff.ptr(q), ff.ptr(k), ff.ptr(v), ff.ptr(o), B, H, KV, Sq, Sk, w,
                                            1 / math.sqrt(128), ff.stream_ptr()))
torch.cuda.synchronize()
print("done")
