#!/usr/bin/env python3
"""Experiment: do the two CFG halves of a DiT forward gain from running as two concurrent
streams?  Times (a) the production Bc = 2 forward (row dedup + closed-form null rows),
(b) a conditional Bc = 1 forward and a null-row Bc = 1 forward back to back on one stream,
(c) the same two forwards on two streams, launched interleaved."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip.config import DiTConfig
from acehip.dit import DiTRuntime
from acehip.weights import synth_dit_weights

dev = torch.device("cuda:0")
cfg = DiTConfig()
T = int(float(os.environ.get("SECONDS", "240")) * 25); S = (T + 1) // 2
W = synth_dit_weights(cfg, seed=0, mode="bench", device=dev, dtype=torch.bfloat16, backend="torch")
rts = []
for _ in range(3):
    rt = DiTRuntime(cfg, 0, max_S=S, max_Bc=2, max_Lenc=641)
    rt.load(W)
    rts.append(rt)
del W
P, A, B = rts
g = torch.Generator(device=dev).manual_seed(0)
enc = torch.randn(1, 641, 2048, device=dev, generator=g).bfloat16()
null = torch.randn(1, 1, 2048, device=dev, generator=g).bfloat16().expand(1, 641, 2048).contiguous()
P.set_condition(torch.cat([enc, null])); P.set_uniform_rows(1)
A.set_condition(enc)
B.set_condition(null); B.set_uniform_rows(0)
xt = torch.randn(1, T, 64, device=dev, generator=g).bfloat16()
ctx = torch.randn(1, T, 128, device=dev, generator=g).bfloat16()
t = torch.tensor([0.75], device=dev)
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
oa = torch.empty(1, T, 64, device=dev, dtype=torch.bfloat16)
ob = torch.empty_like(oa)
op = torch.empty(2, T, 64, device=dev, dtype=torch.bfloat16)


def prod():
    P.forward(xt, ctx, t, out=op)


def seq():
    A.forward(xt, ctx, t, out=oa)
    B.forward(xt, ctx, t, out=ob)


def dual():
    cur = torch.cuda.current_stream()
    s0.wait_stream(cur); s1.wait_stream(cur)
    with torch.cuda.stream(s0):
        A.forward(xt, ctx, t, out=oa)
    with torch.cuda.stream(s1):
        B.forward(xt, ctx, t, out=ob)
    cur.wait_stream(s0); cur.wait_stream(s1)


def bench(f, n=8):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for f in (prod, seq, dual):
    f()
torch.cuda.synchronize()
ref_a, ref_b = oa.clone(), ob.clone()
seq(); torch.cuda.synchronize()
same_seq = torch.equal(oa, ref_a) and torch.equal(ob, ref_b)
res = {"prod": [], "seq": [], "dual": []}
for rd in range(5):
    for name, f in (("prod", prod), ("seq", seq), ("dual", dual)):
        res[name].append(bench(f))
dual(); torch.cuda.synchronize()
print("bit-identical dual vs seq:", torch.equal(oa, ref_a) and torch.equal(ob, ref_b), same_seq)
print("cond rows prod vs A rel:", float((op[0].float() - oa[0].float()).norm() / oa[0].float().norm()))
for k, v in res.items():
    v = sorted(v)
    print(f"{k:5s} ms/forward median {v[len(v) // 2]:.3f} min {v[0]:.3f} all {[round(x, 3) for x in v]}")
