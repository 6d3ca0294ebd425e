#!/usr/bin/env python3
"""Small-M GEMM A/B (turbo / short songs, M = Bc·S = 125 at 10 s turbo): the
weight-streaming skinny kernel at ring depth 2/3/4 against the 128×128 split-K path and
torch (hipBLASLt), weights cold (rotated copies > 600 MB, as in the DiT forward), store
epilogue; interleaved rounds in one process, median of the rounds."""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip import _ffi as ff

dev = torch.device("cuda:0")
M = int(os.environ.get("M", "125"))
shapes = {"swiglu": (12288, 2048), "down": (2048, 6144), "qkv": (4096, 2048), "o": (2048, 2048)}
modes = {"skinny_d2": 102, "skinny_d3": 103, "skinny_d4": 104, "splitk128": 100}
out = {}
for name, (N, K) in shapes.items():
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
    nrot = max(2, int(700e6 // (N * K * 2)))
    Ws = [((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).bfloat16() for _ in range(nrot)]
    ref = A.float() @ Ws[0].float().t()
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    wbytes = N * K * 2 + M * K * 2 + M * N * 2
    times = {k: [] for k in list(modes) + ["torch"]}
    errs = {}
    for k, v in modes.items():
        ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(Ws[0]), K, ff.ptr(C), N, M, N, K, None, 0, v,
                                              ff.stream_ptr()))
        torch.cuda.synchronize()
        errs[k] = round(float((C.float() - ref).norm() / ref.norm()), 5)
    it = [0]
    for rnd in range(5):
        for k in list(modes) + ["torch"]:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 30
            e0.record()
            for _ in range(n):
                W = Ws[it[0] % nrot]
                it[0] += 1
                if k == "torch":
                    torch.matmul(A, W.t(), out=C)
                else:
                    ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(C), N, M, N, K, None, 0,
                                                 modes[k], ff.stream_ptr())
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / n * 1e3)
    row = {}
    for k, ts in times.items():
        us = sorted(ts)[len(ts) // 2]
        row[k] = {"us": round(us, 2), "TB/s": round(wbytes / us * 1e-6, 2), "rel": errs.get(k)}
    out[name] = row
    print(name, f"M={M} N={N} K={K}", json.dumps(row), flush=True)
json.dump(out, open(os.path.join(REPO, "gpurun_out", f"bench_skinny_M{M}.json"), "w"), indent=1)
