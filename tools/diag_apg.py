#!/usr/bin/env python3
"""Diagnose APG multi-chunk mismatches: run the fused step with out_mode=1 (returns the
guided v) and compare stage by stage with the oracle on identical inputs."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip.dit import apg_euler_
from oracle import sampler_oracle as so

dev = torch.device("cuda:0")
for T in (1001, 6000, 512, 257, 256):
    B, C, G = 2, 64, 7.0
    g = torch.Generator().manual_seed(T)
    xt = torch.randn(B, T, C, generator=g).bfloat16()
    ra = torch.zeros(B, T, C, dtype=torch.bfloat16)
    xd, rd = xt.to(dev), ra.to(dev)
    for step, (apply, first) in enumerate([(1, 1), (1, 0), (1, 0)]):
        vt = (torch.randn(2 * B, T, C, generator=g) * (1.0 + step)).bfloat16()
        r0 = rd.cpu()
        vd = xd.clone()
        rr = rd.clone()
        apg_euler_(vt.to(dev), vd, rr, G, 0.0, apply, first, out_mode=1)
        torch.cuda.synchronize()
        cond, unc = vt.chunk(2)
        mom = so.Momentum(); mom.running_average = 0 if first else r0
        v = so.apg(cond, unc, G, mom, dims=(1,))
        got = vd.cpu()
        mm = (got != v)
        print(f"T={T} step={step} ra_equal={torch.equal(rr.cpu(), mom.running_average)} v_mismatch={mm.float().mean().item():.4f}",
              "cols with mismatches:", int(mm.any(dim=1).sum()), "of", B * C,
              "max|d|", (got.float() - v.float()).abs().max().item())
        if mm.any():
            b, t, c = [int(i) for i in mm.nonzero()[0]]
            print("   first mismatch b,t,c", b, t, c, "got", got[b, t, c].item(), "ref", v[b, t, c].item())
            col = mm[b, :, c]
            print("   mismatches in that column:", int(col.sum()), "rows", col.nonzero().flatten()[:10].tolist())
        # advance both with the same Euler step so the next step starts identical
        apg_euler_(vt.to(dev), xd, rd, G, 0.03125, apply, first)
        torch.cuda.synchronize()
