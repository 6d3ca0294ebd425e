#!/usr/bin/env python3
"""RMSNorm+AdaLN rows-per-wave variants at the DiT shape (M = 6000, D = 2048), one process."""
import os, sys, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip import _ffi as ff

dev = torch.device("cuda:0")
M, D, S = 6000, 2048, 3000
x = torch.randn(M, D, device=dev).bfloat16()
w = torch.ones(D, device=dev).bfloat16()
tab = (0.1 * torch.randn(2, 6, D, device=dev)).bfloat16()
out = torch.empty_like(x)
res = {}
for mod in (True, False):
    for r in (1, 2, 4, -2, -4):
        def run():
            ff.check(ff.lib().acehip_rmsnorm_bf16(ff.ptr(x), ff.ptr(w), ff.ptr(tab[:, 0]) if mod else None,
                                                  ff.ptr(tab[:, 1]) if mod else None, 6 * D, S, ff.ptr(out),
                                                  M, D, 1e-6, r, ff.stream_ptr()))
        for _ in range(5): run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50): run()
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 50 * 1e3
        res[f"{'mod' if mod else 'plain'}_R{r}"] = {"us": round(us, 2), "GB/s": round(4 * M * D / us / 1e3, 1)}
print(json.dumps(res))
