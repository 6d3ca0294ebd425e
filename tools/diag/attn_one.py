#!/usr/bin/env python3
"""Run one attention shape a few times (for rocprofv3 counter passes).
usage: attn_one.py <full|band|cross> [S] [reps]"""
import math
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip import _ffi as ff  # noqa: E402

name = sys.argv[1]
S = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
B, H, KV = 2, 16, 8
Sk, w = {"full": (S, -1), "band": (S, 128), "cross": (641, -1)}[name]
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(B, H, S, 128, device=dev, generator=g).bfloat16()
k = torch.randn(B, KV, Sk, 128, device=dev, generator=g).bfloat16()
v = torch.randn(B, KV, Sk, 128, device=dev, generator=g).bfloat16()
o = torch.empty(B, S, H * 128, device=dev, dtype=torch.bfloat16)
f = ff.lib().acehip_attention_bf16
for _ in range(reps):
    assert f(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, KV, S, Sk, w, 1 / math.sqrt(128),
             ff.stream_ptr()) == 0
torch.cuda.synchronize()
print("ok", name, S)
