import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd"), os.path.join(REPO, "tests")]
import torch
from test_gpu_fused import _headpost_ref
from oracle import dit_oracle
from acehip import _ffi as ff
dev = torch.device("cuda:0")
B, S, nq, nk, nv, K = 2, 300, 4, 2, 2, 256
g = torch.Generator().manual_seed(1)
N = (nq + nk + nv) * 128
A = torch.randn(B * S, K, generator=g).bfloat16()
W = (torch.randn(N, K, generator=g) * 0.05).bfloat16()
qw = torch.ones(128).bfloat16(); kw = torch.ones(128).bfloat16()
for rope in (False, True):
    cos, sin = dit_oracle.rope_tables(S, 128, 1e6, torch.bfloat16) if rope else (None, None)
    if rope: cos, sin = cos[0].contiguous(), sin[0].contiguous()
    d = lambda t: None if t is None else t.to(dev)
    Ad, Wd = d(A), d(W)
    qwd, kwd, cosd, sind = d(qw), d(kw), d(cos), d(sin)   # kept alive across the launch
    q = torch.zeros(B, nq, S, 128, dtype=torch.bfloat16, device=dev)
    k = torch.zeros(B, nk, S, 128, dtype=torch.bfloat16, device=dev)
    v = torch.zeros(B, nv, S, 128, dtype=torch.bfloat16, device=dev)
    ff.check(ff.lib().acehip_gemm_headpost_bf16(ff.ptr(Ad), K, ff.ptr(Wd), K, B, S, nq, nk, nv, ff.ptr(qwd), ff.ptr(kwd),
        ff.ptr(cosd), ff.ptr(sind), 1e-6, ff.ptr(q), ff.ptr(k), ff.ptr(v), ff.stream_ptr()))
    C = torch.empty(B * S, N, dtype=torch.bfloat16, device=dev)
    ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(Ad), K, ff.ptr(Wd), K, ff.ptr(C), N, B * S, N, K, None, 0, 8, ff.stream_ptr()))
    torch.cuda.synchronize()
    rq, rk, rv = _headpost_ref(C.cpu(), B, S, nq, nk, nv, qw, kw, cos, sin, 1e-6)
    for nm, got, ref in (("q", q, rq), ("k", k, rk), ("v", v, rv)):
        got = got.cpu().float(); ref = ref.float()
        bad = (got - ref).abs() > 0.02 * ref.abs().max()
        print(rope, nm, "bad frac", bad.float().mean().item())
        if bad.any():
            idx = bad.nonzero()
            print("  first bad idx", idx[:5].tolist(), "rows bad per (b,h):", bad.any(-1).sum(-1).tolist())
            print("  cols bad:", bad.any(0).any(0).any(0).nonzero().flatten()[:40].tolist())
            b_, h_, s_, c_ = idx[0].tolist()
            print("  got", got[b_, h_, s_, :8].tolist(), "\n  ref", ref[b_, h_, s_, :8].tolist())
            print("  zero frac got", (got == 0).float().mean().item())
