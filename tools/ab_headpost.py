#!/usr/bin/env python3
"""Interleaved in-process A/B of the fused head-post GEMM (QKV: q/k RMSNorm + RoPE +
head-major scatter; cross-Q: q norm only) between the working-tree library and
alternative builds (tools/ab_build.sh).  usage: ab_headpost.py tools/ab/libacehip_ref.so"""
import ctypes, json, os, statistics, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip import _ffi as ff  # noqa: E402

dev = torch.device("cuda:0")
B, S, K = 2, 3000, 2048
M = B * S
A = torch.randn(M, K, device=dev).bfloat16()
cos = torch.randn(S, 128, device=dev).bfloat16(); sin = torch.randn(S, 128, device=dev).bfloat16()
qw = (1 + 0.1 * torch.randn(128, device=dev)).bfloat16()
libs = [("tree", ff.lib().acehip_gemm_headpost_bf16)]
for p in sys.argv[1:]:
    lib = ctypes.CDLL(os.path.abspath(p))
    f = lib.acehip_gemm_headpost_bf16
    f.argtypes, f.restype = ff.lib().acehip_gemm_headpost_bf16.argtypes, ctypes.c_int
    libs.append((os.path.basename(p), f))
res = {}
for name, (nq, nk, nv, rope, bb) in {"qkv": (16, 8, 8, True, 2), "crossq": (16, 0, 0, False, 1)}.items():
    Bq = bb
    Mq = Bq * S
    N = (nq + nk + nv) * 128
    W = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
    outs, times = {}, {n: [] for n, _ in libs}
    for lname, f in libs:
        q = torch.zeros(Bq, max(nq, 1), S, 128, device=dev, dtype=torch.bfloat16)
        k = torch.zeros(Bq, max(nk, 1), S, 128, device=dev, dtype=torch.bfloat16)
        v = torch.zeros(Bq, max(nv, 1), S, 128, device=dev, dtype=torch.bfloat16)
        call = lambda f=f, q=q, k=k, v=v: ff.check(f(ff.ptr(A), K, ff.ptr(W), K, Bq, S, nq, nk, nv, ff.ptr(qw),
                                                    ff.ptr(qw), ff.ptr(cos) if rope else None,
                                                    ff.ptr(sin) if rope else None, 1e-6, ff.ptr(q), ff.ptr(k),
                                                    ff.ptr(v), ff.stream_ptr()))
        call()
        torch.cuda.synchronize()
        outs[lname] = (q.clone(), k.clone(), v.clone(), call)
    for _ in range(5):
        for lname, _f in libs:
            call = outs[lname][3]
            for _ in range(3): call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20): call()
            e1.record(); torch.cuda.synchronize()
            times[lname].append(e0.elapsed_time(e1) / 20 * 1e3)
    base = outs["tree"]
    res[name] = {ln: {"us": round(statistics.median(t), 1),
                      "maxdiff": max(float((a.float() - b.float()).abs().max()) for a, b in zip(outs[ln][:3], base[:3]))}
                 for ln, t in times.items()}
    print(name, res[name], flush=True)
print(json.dumps(res))
