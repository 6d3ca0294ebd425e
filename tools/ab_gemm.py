#!/usr/bin/env python3
"""Interleaved in-process A/B of the GEMM between the working-tree library and
alternative builds (tools/ab_build.sh) on the DiT shapes, production variant
choice (acehip_gemm_bf16_ex with the picked variant) and epilogues.

usage: ab_gemm.py tools/ab/libacehip_ref.so [...]
"""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip import _ffi as ff  # noqa: E402

dev = torch.device("cuda:0")
# name: (M, N, K, epi, variant)  — epi 0 store, 3 SwiGLU; variants as the cost model picks them
SHAPES = {"swiglu": (6000, 12288, 2048, 3, 7), "down": (6000, 2048, 6144, 2, 8), "qkv": (6000, 4096, 2048, 0, 8),
          "o": (6000, 2048, 2048, 2, 8), "o_half": (3000, 2048, 2048, 2, 13), "crossq": (3000, 2048, 2048, 0, 13),
          "swiglu_prod": (6000, 12288, 2048, 3, -1)}   # -1: the production dispatch (tail split included)


def load(path):
    if path is None:
        return "tree", ff.lib().acehip_gemm_bf16_ex
    lib = ctypes.CDLL(os.path.abspath(path))
    f = lib.acehip_gemm_bf16_ex
    P, I = ctypes.c_void_p, ctypes.c_int
    f.argtypes = [P, I, P, I, P, I, I, I, I, P, I, I, P]
    f.restype = I
    return os.path.basename(path), f


libs = [load(None)] + [load(p) for p in sys.argv[1:]]
# AB_VARIANT forces one variant for every shape (A/B of a kernel's schedule builds)
if os.environ.get("AB_VARIANT"):
    SHAPES = {k: v[:4] + (int(os.environ["AB_VARIANT"]),) for k, v in SHAPES.items()}
# AB_VARIANTS=v1,v2,...: every listed variant of the working-tree library as its own arm
EXTRA_VARIANTS = [int(v) for v in os.environ.get("AB_VARIANTS", "").split(",") if v]
# AB_KNOBS=NAME=VAL;...: the working-tree library with one switch set, as its own arm (the
# library reads its switches once: set + acehip_reload_knobs around that arm's launches)
EXTRA_KNOBS = [kv for kv in os.environ.get("AB_KNOBS", "").split(";") if kv]


def knob(label):
    if label.startswith("tree_") and "=" in label:
        k, v = label[5:].split("=", 1)
        os.environ[k] = v
        ff.reload_knobs()
        return k
    return None


def unknob(k):
    if k:
        os.environ.pop(k)
        ff.reload_knobs()
if os.environ.get("SHAPES"):
    SHAPES = {k: v for k, v in SHAPES.items() if k in os.environ["SHAPES"].split(",")}
res = {}
for name, (M, N, K, epi, var) in SHAPES.items():
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
    # weights rotated through > 600 MB of copies so W comes from HBM as in the DiT
    nrot = max(1, int(600e6 // (N * K * 2)))
    Ws = [((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).bfloat16() for _ in range(min(nrot, 4))]
    Ws += [Ws[i % len(Ws)].clone() for i in range(nrot - len(Ws))]
    ldc = N // 2 if epi == 3 else N
    # arms: (label, entry point, variant) — every library at the shape's variant, plus the
    # working tree's AB_VARIANTS
    arms = [(ln, f, var) for ln, f in libs] + [(f"tree_v{v}", libs[0][1], v) for v in EXTRA_VARIANTS]
    arms += [(f"tree_{kv}", libs[0][1], var) for kv in EXTRA_KNOBS]
    outs = {}
    times = {ln: [] for ln, _, _ in arms}
    rot = [0]

    def run(f, v, C):
        W = Ws[rot[0] % nrot]
        rot[0] += 1
        assert f(A.data_ptr(), K, W.data_ptr(), K, C.data_ptr(), ldc, M, N, K, None, epi, v,
                 ff.stream_ptr().value) == 0

    for ln, f, v in arms:
        C = torch.zeros(M, ldc, device=dev, dtype=torch.bfloat16)   # the residual of epi 2
        rot[0] = 0
        kk = knob(ln)
        run(f, v, C)
        torch.cuda.synchronize()
        unknob(kk)
        outs[ln] = C.float()
    for _ in range(5):
        for ln, f, v in arms:
            C = torch.zeros(M, ldc, device=dev, dtype=torch.bfloat16)
            kk = knob(ln)
            for _ in range(3):
                run(f, v, C)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 20
            e0.record()
            for _ in range(n):
                run(f, v, C)
            e1.record()
            torch.cuda.synchronize()
            unknob(kk)
            times[ln].append(e0.elapsed_time(e1) / n * 1e3)
    # hipBLASLt (torch.matmul, plain store, no epilogue) on the same box for reference
    Wts = [w.t() for w in Ws]
    for i in range(3):
        torch.matmul(A, Wts[i % nrot])
    tt = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(20):
            torch.matmul(A, Wts[i % nrot])
        e1.record()
        torch.cuda.synchronize()
        tt.append(e0.elapsed_time(e1) / 20 * 1e3)
    fl = 2.0 * M * N * K
    row = {"torch(hipBLASLt)": {"us": round(statistics.median(tt), 1),
                                "tflops": round(fl / statistics.median(tt) * 1e-6, 1)}}
    for ln in times:
        us = statistics.median(times[ln])
        d = float((outs[ln] - outs["tree"]).abs().max())
        row[ln] = {"us": round(us, 1), "tflops": round(fl / us * 1e-6, 1), "maxdiff_vs_tree": d}
    res[name] = row
    print(name, json.dumps(row), flush=True)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(REPO, "gpurun_out", "ab_gemm.json"), "w"), indent=1)
