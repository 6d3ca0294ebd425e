#!/usr/bin/env python3
"""GEMM variant micro-benchmark on the DiT shapes (M = Bc·S = 6000 at 240 s)."""
import os, sys, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip import _ffi as ff

dev = torch.device("cuda:0")
shapes = {"swiglu": (6000, 12288, 2048), "down": (6000, 2048, 6144), "qkv": (6000, 4096, 2048),
          "o": (6000, 2048, 2048), "o_half": (3000, 2048, 2048), "qkv_half": (3000, 4096, 2048), "crossq": (3000, 2048, 2048), "eq_k6144": (8192, 2048, 6144), "eq_k2048": (8192, 2048, 2048), "vae_k7_c128": (46080, 128, 896), "vae_k7_c512": (360000 // 4, 512, 3584),
          # stream-K what-if probes: one round of 256² tiles at a given K-tile count
          "r256_k2048": (4096, 4096, 2048), "r128_k1024": (2048, 4096, 1024), "r256_k4608": (4096, 4096, 4608),
          "r256_k1536": (4096, 4096, 1536)}
variants = [int(v) for v in os.environ.get("VARIANTS", "0,4,6,7,8").split(",")]
# COLD=1: rotate through enough weight copies (> 512 MB) that W comes from HBM
# every launch, as in the DiT forward (1.2 GB of weights per step, MALL 256 MB)
COLD = os.environ.get("COLD", "0") == "1"
only = os.environ.get("SHAPES")
if only:
    shapes = {k: v for k, v in shapes.items() if k in only.split(",")}
res = {}
for name, (M, N, K) in shapes.items():
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
    W = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).bfloat16()
    ref = (A.float() @ W.float().t())
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    nrot = max(1, int(600e6 // (N * K * 2))) if COLD else 1
    Ws = [W] + [W.clone() for _ in range(nrot - 1)]
    rot = [0]
    fl = 2.0 * M * N * K
    row = {}
    times = {}
    # ROUNDS > 1: the variants are timed in interleaved rounds (v1 v2 … v1 v2 …) and the
    # median per variant is reported, so clock drift over the run does not favour one
    for rd in range(int(os.environ.get("ROUNDS", "1"))):
      for v in variants:
        if v in (7, 8, 11) and N % 256:
            continue
        def run():
            Wr = Ws[rot[0] % nrot]
            rot[0] += 1
            ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(Wr), K, ff.ptr(C), N, M, N, K, None, 0, v,
                                                  ff.stream_ptr()))
        rot[0] = 0
        run(); torch.cuda.synchronize()
        err = float((C.float() - ref).norm() / ref.norm())
        for _ in range(3): run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n): run()
        e1.record(); torch.cuda.synchronize()
        times.setdefault(v, []).append(e0.elapsed_time(e1) / n * 1e3)
        us = sorted(times[v])[len(times[v]) // 2]
        row[f"v{v}"] = {"us": round(us, 1), "tflops": round(fl / us * 1e-6, 1), "rel": round(err, 5)}
    Wts = [w.t() for w in Ws]
    for i in range(3): torch.matmul(A, Wts[i % nrot])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(20): torch.matmul(A, Wts[i % nrot])
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    row["torch(hipBLASLt)"] = {"us": round(us, 1), "tflops": round(fl / us * 1e-6, 1)}
    res[name] = row
    print(name, json.dumps(row), flush=True)
