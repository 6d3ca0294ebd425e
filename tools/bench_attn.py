#!/usr/bin/env python3
"""Attention micro-benchmark at the DiT's shapes (240 s: Bc=2, H=16, KV=8,
S=3000; cross Lenc=641), interleaved A/B between the working-tree library and
any number of alternative builds (tools/ab_build.sh) in ONE process.

usage: bench_attn.py [tools/ab/libacehip_ref.so ...]
AB_ENV="VAR=VAL,..." is put into the environment after the tree library's first call, so the
alternative builds (which read their knobs lazily at their own first call) see it and the tree
does not: a knob A/B with a copy of the tree's own library.
"""
import ctypes
import json
import math
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip import _ffi as ff  # noqa: E402

dev = torch.device("cuda:0")
S = int(os.environ.get("ATTN_S", "3000"))
B0 = int(os.environ.get("ATTN_B", "2"))
SHAPES = {"full": (B0, 16, 8, S, S, -1), "band": (B0, 16, 8, S, S, 128), "cross": (B0, 16, 8, S, 641, -1),
          "cross1": (1, 16, 8, S, 641, -1)}
if os.environ.get("SHAPES"):
    SHAPES = {k: v for k, v in SHAPES.items() if k in os.environ["SHAPES"].split(",")}


def flops(B, H, Sq, Sk, w):
    if w < 0:
        pairs = Sq * Sk
    else:
        pairs = sum(min(Sk, i + w + 1) - max(0, i - w) for i in range(Sq))
    return 4.0 * pairs * 128 * H * B


def load(path):
    if path is None:
        return "tree", ff.lib().acehip_attention_bf16
    lib = ctypes.CDLL(os.path.abspath(path))
    f = lib.acehip_attention_bf16
    P, I = ctypes.c_void_p, ctypes.c_int
    f.argtypes = [P, P, P, P, I, I, I, I, I, I, ctypes.c_float, P]
    f.restype = I
    return os.path.basename(path), f


libs = [load(None)] + [load(p) for p in sys.argv[1:]]
res = {}
for name, (B, H, KV, Sq, Sk, w) in SHAPES.items():
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B, H, Sq, 128, device=dev, generator=g).bfloat16()
    k = torch.randn(B, KV, Sk, 128, device=dev, generator=g).bfloat16()
    v = torch.randn(B, KV, Sk, 128, device=dev, generator=g).bfloat16()
    outs = {}
    times = {ln: [] for ln, _ in libs}
    for ln, f in libs:
        o = torch.empty(B, Sq, H * 128, device=dev, dtype=torch.bfloat16)
        assert f(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, KV, Sq, Sk, w,
                 1 / math.sqrt(128), ff.stream_ptr()) == 0
        torch.cuda.synchronize()
        outs[ln] = o.float()
        if ln == "tree" and os.environ.get("AB_ENV"):
            for kv in os.environ.pop("AB_ENV").split(","):
                os.environ[kv.split("=")[0]] = kv.split("=", 1)[1]
    for _ in range(5):                       # interleaved rounds
        for ln, f in libs:
            o = torch.empty(B, Sq, H * 128, device=dev, dtype=torch.bfloat16)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, KV, Sq, Sk, w,
                  1 / math.sqrt(128), ff.stream_ptr())
            e1.record()
            torch.cuda.synchronize()
            times[ln].append(e0.elapsed_time(e1) / 10 * 1e3)
    fl = flops(B, H, Sq, Sk, w)
    base = outs[libs[0][0]]
    row = {}
    for ln, _ in libs:
        us = statistics.median(times[ln])
        row[ln] = {"us": round(us, 1), "tflops": round(fl / us * 1e-6, 1),
                   "rel_vs_tree": round(float((outs[ln] - base).norm() / base.norm()), 5)}
    res[name] = row
    print(name, json.dumps(row), flush=True)
