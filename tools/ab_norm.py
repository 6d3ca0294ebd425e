#!/usr/bin/env python3
"""RMSNorm+AdaLN at the DiT shape (M = 6000, D = 2048): the working-tree library against other
builds (tools/ab_build.sh), interleaved rounds in one process, medians; outputs compared.
usage: ab_norm.py tools/ab/libacehip_head.so"""
import ctypes, json, os, statistics, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip import _ffi as ff  # noqa: E402

dev = torch.device("cuda:0")
M, D, S = 6000, 2048, 3000
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(M, D, device=dev, generator=g).bfloat16()
w = (1 + 0.1 * torch.randn(D, device=dev, generator=g)).bfloat16()
tab = (0.1 * torch.randn(2, 6, D, device=dev, generator=g)).bfloat16()
libs = [("tree", ff.lib().acehip_rmsnorm_bf16)]
RPW = [int(r) for r in os.environ.get("RPW", "0").split(",")]   # rows-per-wave variants of the tree
for p in sys.argv[1:]:
    f = ctypes.CDLL(os.path.abspath(p)).acehip_rmsnorm_bf16
    f.argtypes, f.restype = ff.lib().acehip_rmsnorm_bf16.argtypes, ctypes.c_int
    libs.append((os.path.basename(p), f))
res = {}
for mod in (True, False):
    arms = [(ln, f, 0) for ln, f in libs] + [(f"tree_R{r}", libs[0][1], r) for r in RPW if r]
    outs, times = {}, {n: [] for n, _, _ in arms}
    for ln, f, rr in arms:
        out = torch.empty_like(x)
        run = lambda f=f, out=out, rr=rr: ff.check(f(ff.ptr(x), ff.ptr(w), ff.ptr(tab[:, 0]) if mod else None,
                                                     ff.ptr(tab[:, 1]) if mod else None, 6 * D, S, ff.ptr(out), M,
                                                     D, 1e-6, rr, ff.stream_ptr()))
        run()
        torch.cuda.synchronize()
        outs[ln] = (out.clone(), run)
    for _ in range(7):
        for ln, _f, _r in arms:
            run = outs[ln][1]
            for _ in range(3): run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50): run()
            e1.record(); torch.cuda.synchronize()
            times[ln].append(e0.elapsed_time(e1) / 50 * 1e3)
    ref = outs["tree"][0].float()
    res["mod" if mod else "plain"] = {ln: {"us": round(statistics.median(t), 2),
                                           "mismatch_frac": float((outs[ln][0].float() != ref).float().mean())}
                                      for ln, t in times.items()}
    print("mod" if mod else "plain", res["mod" if mod else "plain"], flush=True)
print(json.dumps(res))
