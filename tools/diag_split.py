#!/usr/bin/env python3
"""Attention tail-split parity for several builds of libacehip (tree + tools/ab/*.so given on
the command line): the 24-unit split case of tests/test_gpu_dit.py::test_attention_tail_split
(ACEHIP_ATTN_CUS = 16/18/20 → 2/3/4-way splits) and a no-split full / band case, vs fp32 torch."""
import ctypes, math, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip import _ffi as ff

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
    return (s.softmax(-1) @ vv).transpose(1, 2).reshape(q.shape[0], Sq, -1)


libs = [("tree", ff.lib().acehip_attention_bf16)]
for p in sys.argv[1:]:
    f = ctypes.CDLL(os.path.abspath(p)).acehip_attention_bf16
    P, I = ctypes.c_void_p, ctypes.c_int
    f.argtypes = [P, P, P, P, I, I, I, I, I, I, ctypes.c_float, P]
    f.restype = I
    libs.append((os.path.basename(p), f))
B, H, KV, Sq, Sk = 2, 4, 2, 700, 1600
g = torch.Generator(device="cpu").manual_seed(1)
q = torch.randn(B, H, Sq, 128, generator=g).to(dev, torch.bfloat16)
k = torch.randn(B, KV, Sk, 128, generator=g).to(dev, torch.bfloat16)
v = torch.randn(B, KV, Sk, 128, generator=g).to(dev, torch.bfloat16)
for pw in ("0", "7"):
    os.environ["ACEHIP_ATTN_PW"] = pw
    for cus in ("16", "20", "256"):
        os.environ["ACEHIP_ATTN_CUS"] = cus
        for w in (-1, 128):
            r = ref(q, k, v, w)
            row = []
            for name, f in libs:
                o = torch.empty(B, Sq, H * 128, device=dev, dtype=torch.bfloat16)
                rc = f(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, KV, Sq, Sk, w, 1 / math.sqrt(128),
                       ff.stream_ptr())
                torch.cuda.synchronize()
                row.append(f"{name}={float((o.float() - r).norm() / r.norm()):.4f}(rc{rc})")
            print(f"pw={pw} cus={cus} w={w}: " + " ".join(row), flush=True)
