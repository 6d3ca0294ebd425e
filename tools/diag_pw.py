#!/usr/bin/env python3
"""attn_pw_kernel diagnostics: rel-L2 vs an fp32 reference and vs the 32-row kernel
(ACEHIP_ATTN_PW=0) on small shapes, with and without the tail split."""
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip import _ffi as ff  # noqa: E402

dev = torch.device("cuda:0")


def ref(q, k, v, window):
    Sq, Sk = q.shape[2], k.shape[2]
    rep = q.shape[1] // k.shape[1]
    kk = k.float().repeat_interleave(rep, 1)
    vv = v.float().repeat_interleave(rep, 1)
    s = (q.float() @ kk.transpose(2, 3)) / math.sqrt(128)
    if window >= 0:
        i = torch.arange(Sq, device=q.device)[:, None]
        j = torch.arange(Sk, device=q.device)[None, :]
        s = s.masked_fill((i - j).abs() > window, float("-inf"))
    return (torch.softmax(s, -1) @ vv).transpose(1, 2).reshape(q.shape[0], Sq, -1)


def run(q, k, v, window):
    B, H, Sq, _ = q.shape
    o = torch.empty(B, Sq, H * 128, device=dev, dtype=torch.bfloat16)
    ff.check(ff.lib().acehip_attention_bf16(ff.ptr(q), ff.ptr(k), ff.ptr(v), ff.ptr(o), B, H, k.shape[1], Sq,
                                            k.shape[2], window, 1 / math.sqrt(128), ff.stream_ptr()))
    torch.cuda.synchronize()
    return o.float()


cases = [(1, 2, 1, 128, 64, -1), (1, 2, 1, 128, 128, -1), (1, 2, 1, 128, 640, -1), (2, 4, 2, 700, 1600, -1),
         (1, 2, 1, 300, 300, 128), (2, 4, 2, 700, 641, -1), (1, 2, 1, 1000, 1000, 128)]
for cus in ["", "16"]:
    if cus:
        os.environ["ACEHIP_ATTN_CUS"] = cus
    for (B, H, KV, Sq, Sk, w) in cases:
        g = torch.Generator(device="cpu").manual_seed(Sq + Sk)
        q = torch.randn(B, H, Sq, 128, generator=g).to(dev, torch.bfloat16)
        k = torch.randn(B, KV, Sk, 128, generator=g).to(dev, torch.bfloat16)
        v = torch.randn(B, KV, Sk, 128, generator=g).to(dev, torch.bfloat16)
        r = ref(q, k, v, w)
        os.environ["ACEHIP_ATTN_PW"] = "7"
        a = run(q, k, v, w)
        os.environ["ACEHIP_ATTN_PW"] = "0"
        b = run(q, k, v, w)
        e1 = float((a - r).norm() / r.norm())
        e0 = float((b - r).norm() / r.norm())
        # per-row-block error map for the pw kernel
        rowerr = ((a - r).norm(dim=-1) / r.norm(dim=-1).clamp_min(1e-9))[0]
        bad = (rowerr > 0.05).nonzero().flatten().tolist()
        print(f"cus={cus or 'dev'} B{B} H{H} KV{KV} Sq{Sq} Sk{Sk} w{w}: pw {e1:.4g} old {e0:.4g} "
              f"bad rows {len(bad)} first {bad[:8]} a[0,0,:4]={a[0,0,:4].tolist()} r={r[0,0,:4].tolist()}", flush=True)
