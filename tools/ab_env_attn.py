#!/usr/bin/env python3
"""Attention A/B over environment knobs in ONE process (the library reads them per call):
interleaved timing of every setting on the DiT shapes.

usage: ab_env_attn.py 'NAME=VAL[,NAME=VAL]' ['...' ...]   (the first setting is the baseline)"""
import math
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip._ffi import reload_knobs  # noqa: E402  (the library reads its switches once)
from acehip import _ffi as ff  # noqa: E402

dev = torch.device("cuda:0")
S = int(os.environ.get("ATTN_S", "3000"))
SHAPES = {"full": (2, 16, 8, S, S, -1), "band": (2, 16, 8, S, S, 128), "cross1": (1, 16, 8, S, 641, -1)}
if os.environ.get("SHAPES"):
    SHAPES = {k: v for k, v in SHAPES.items() if k in os.environ["SHAPES"].split(",")}
settings = [dict(kv.split("=") for kv in a.split(",") if kv) for a in sys.argv[1:]] or [{}]


def call(q, k, v, o, B, H, KV, Sq, Sk, w):
    ff.check(ff.lib().acehip_attention_bf16(ff.ptr(q), ff.ptr(k), ff.ptr(v), ff.ptr(o), B, H, KV, Sq, Sk, w,
                                            1 / math.sqrt(128), ff.stream_ptr()))


for name, (B, H, KV, Sq, Sk, w) in SHAPES.items():
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B, H, Sq, 128, device=dev, generator=g).bfloat16()
    k = torch.randn(B, KV, Sk, 128, device=dev, generator=g).bfloat16()
    v = torch.randn(B, KV, Sk, 128, device=dev, generator=g).bfloat16()
    o = torch.empty(B, Sq, H * 128, device=dev, dtype=torch.bfloat16)
    times = [[] for _ in settings]
    outs = []
    for i, st in enumerate(settings):
        os.environ.update(st)
        reload_knobs()
        call(q, k, v, o, B, H, KV, Sq, Sk, w)
        torch.cuda.synchronize()
        outs.append(o.float().clone())
        for kk in st:
            os.environ.pop(kk)
            reload_knobs()
    for _ in range(7):
        for i, st in enumerate(settings):
            os.environ.update(st)
            reload_knobs()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                call(q, k, v, o, B, H, KV, Sq, Sk, w)
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / 10 * 1e3)
            for kk in st:
                os.environ.pop(kk)
                reload_knobs()
    row = []
    for i, st in enumerate(settings):
        rel = float((outs[i] - outs[0]).norm() / outs[0].norm())
        row.append(f"{','.join(f'{a}={b}' for a, b in st.items()) or 'default'}: {statistics.median(times[i]):.1f} us"
                   f" (rel {rel:.1e})")
    print(name, " | ".join(row), flush=True)
