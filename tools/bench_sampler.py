#!/usr/bin/env python3
"""One APG+Euler sampler step (the three launches) at the 240 s song shape (B = 1, T = 6000, C = 64)."""
import os, sys, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip.dit import apg_euler_

dev = torch.device("cuda:0")
B, T, C = 1, 6000, 64
vt = torch.randn(2 * B, T, C, device=dev).bfloat16()
xt = torch.randn(B, T, C, device=dev).bfloat16()
ra = torch.zeros_like(xt)
res = {}
for apply in (1, 0):
    for _ in range(5):
        apg_euler_(vt, xt, ra, 7.0, 0.01, apply, 0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        apg_euler_(vt, xt, ra, 7.0, 0.01, apply, 0)
    e1.record()
    torch.cuda.synchronize()
    res["apg" if apply else "euler"] = {"us_per_step": round(e0.elapsed_time(e1) / 100 * 1e3, 2)}
print(json.dumps(res))
