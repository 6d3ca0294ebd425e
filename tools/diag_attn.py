"""Attention kernel diagnostics: V = one-hot columns exposes P directly."""
import math, sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "ace-step-1.5_amd")]
import torch
from acehip import _ffi as ff
dev = torch.device("cuda:0")

def run(q, k, v, window=-1):
    B, H, Sq, _ = q.shape; KV, Sk = k.shape[1], k.shape[2]
    o = torch.zeros(B, Sq, H * 128, device=dev, dtype=torch.bfloat16)
    ff.check(ff.lib().acehip_attention_bf16(ff.ptr(q), ff.ptr(k), ff.ptr(v), ff.ptr(o), B, H, KV, Sq, Sk, window, 1/math.sqrt(128), ff.stream_ptr()))
    torch.cuda.synchronize()
    return o.view(B, Sq, H, 128).transpose(1, 2).float()

torch.manual_seed(0)
Sq, Sk = 32, 64
# 1) uniform P: Q=K=0 → O = mean(V)
q = torch.zeros(1, 1, Sq, 128, device=dev, dtype=torch.bfloat16)
k = torch.zeros(1, 1, Sk, 128, device=dev, dtype=torch.bfloat16)
v = torch.randn(1, 1, Sk, 128, device=dev).bfloat16()
o = run(q, k, v)
print("uniform: max|O - mean V| =", (o[0, 0] - v[0, 0].float().mean(0)).abs().max().item())
# 2) V one-hot: V[key][d] = (d == key) → O[q][d] = P[q][d]
v = torch.zeros(1, 1, Sk, 128, device=dev)
v[0, 0, torch.arange(Sk), torch.arange(Sk)] = 1
v = v.bfloat16()
q = torch.randn(1, 1, Sq, 128, device=dev).bfloat16(); k = torch.randn(1, 1, Sk, 128, device=dev).bfloat16()
o = run(q, k, v)[0, 0, :, :Sk]
p = torch.softmax(q[0, 0].float() @ k[0, 0].float().t() / math.sqrt(128), -1)
print("P err", (o - p).abs().max().item())
# find permutation: for each column d of O, which column of P matches best
corr = (o.t() @ p) / (o.norm(dim=0)[:, None] * p.norm(dim=0)[None, :] + 1e-9)
best = corr.argmax(1).tolist()
print("col map O->P:", best)
rowcorr = (o @ p.t()) / (o.norm(dim=1)[:, None] * p.norm(dim=1)[None, :] + 1e-9)
print("row map O->P:", rowcorr.argmax(1).tolist())
print("O[0,:16]", [round(x, 3) for x in o[0, :16].tolist()])
print("P[0,:16]", [round(x, 3) for x in p[0, :16].tolist()])
