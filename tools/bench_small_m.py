#!/usr/bin/env python3
"""Small-M GEMM A/B at the turbo / short-song shapes (M = Bc·S = 125 at 10 s turbo): the
production dispatch (64-column split-K + its epilogue launch; SwiGLU on whole-K 128×64 tiles
with helper waves, variant 17) against 128-column split-K tiles (ACEHIP_SPLITK_BN=128) and
the whole-K tiles without helpers (variant 16),
cold weights (rotated copies > 600 MB), interleaved rounds in one process, medians."""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip import _ffi as ff  # noqa: E402

dev = torch.device("cuda:0")
M = int(os.environ.get("M", "125"))
# name: (N, K, epi)  epi 0 store, 2 residual (C += A·Wᵀ), 3 SwiGLU (C[M][N/2])
shapes = {"swiglu": (12288, 2048, 3), "down": (2048, 6144, 2), "qkv": (4096, 2048, 0), "o": (2048, 2048, 2)}
cases = {"prod": (-1, {}), "bn128": (-1, {"ACEHIP_SPLITK_BN": "128"}), "v16": (16, {}), "v17": (17, {})}
if os.environ.get("SHAPES"):
    shapes = {k: v for k, v in shapes.items() if k in os.environ["SHAPES"].split(",")}
if os.environ.get("CASES"):        # extra env cases: "name:K=V+K=V;name2:K=V"
    for item in os.environ["CASES"].split(";"):
        nm, kv = item.split(":")
        cases[nm] = (-1, dict(x.split("=") for x in kv.split("+")))
out = {}
for name, (N, K, epi) in shapes.items():
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
    nrot = max(2, int(700e6 // (N * K * 2)))
    Ws = [((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).bfloat16() for _ in range(nrot)]
    nout = N // 2 if epi == 3 else N
    C0 = (torch.rand(M, nout, device=dev, generator=g) * 2 - 1).bfloat16()
    C = C0.clone()
    wbytes = N * K * 2 + M * K * 2 + M * nout * 2 * (2 if epi == 2 else 1)
    mycases = {k: v for k, v in cases.items() if epi == 3 or not k.startswith("v")}
    outs = {}

    def run(k, W):
        var, env = mycases[k]
        return ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(C), nout, M, N, K, None, epi, var,
                                            ff.stream_ptr())

    def setenv(k, on):
        # the library reads its switches once: set / clear the case's, then reload
        env = mycases[k][1]
        for kk, vv in env.items():
            if on:
                os.environ[kk] = vv
            else:
                os.environ.pop(kk)
        if env:
            ff.reload_knobs()
    for k in mycases:
        C.copy_(C0)
        setenv(k, True)
        ff.check(run(k, Ws[0]))
        torch.cuda.synchronize()
        setenv(k, False)
        outs[k] = C.float().clone()
    ref = outs["prod"]
    times = {k: [] for k in mycases}
    it = 0
    for rnd in range(5):
        for k in mycases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 30
            setenv(k, True)
            e0.record()
            for _ in range(n):
                run(k, Ws[it % nrot])
                it += 1
            e1.record()
            torch.cuda.synchronize()
            setenv(k, False)
            times[k].append(e0.elapsed_time(e1) / n * 1e3)
    row = {}
    for k, ts in times.items():
        us = sorted(ts)[len(ts) // 2]
        d = (outs[k] - ref).norm() / ref.norm() if epi != 2 else (outs[k] - ref).norm() / (ref - C0.float()).norm()
        row[k] = {"us": round(us, 2), "TB/s": round(wbytes / us * 1e-6, 2), "rel_vs_prod": round(float(d), 5)}
    out[name] = row
    print(name, f"M={M} N={N} K={K}", json.dumps(row), flush=True)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(REPO, "gpurun_out", f"bench_small_m_M{M}.json"), "w"), indent=1)
