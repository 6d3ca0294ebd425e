"""GPU parity of the fused epilogues and the row-norm kernel against the CPU
oracle's restatement of the reference ops:
  * acehip_gemm_headpost_bf16 — q/k/v projection with Qwen3RMSNorm per head,
    rotate-half RoPE and the head-major scatter fused into the GEMM epilogue
    (reference base:300-345) vs GEMM + oracle.rms_norm + oracle RoPE;
  * acehip_rmsnorm_bf16 — Qwen3RMSNorm + AdaLN modulation (base:499,530,1496),
    every rows-per-wave variant, batch boundaries that split a wave's rows.
Tolerance: the kernels reproduce each bf16 rounding of the torch op sequence,
so they differ from the oracle only where fp32 reduction order flips a bf16
rounding — ≤ 1e-3 of elements, rel-L2 ≤ 2e-3."""
import pytest
import torch

from conftest import rel_l2
from oracle import dit_oracle

pytestmark = pytest.mark.gpu


def _ff():
    from acehip import _ffi
    return _ffi


def _headpost_ref(C, B, S, nq, nk, nv, qw, kw, cos, sin, eps):
    """oracle: split rows [B*S, N] into heads, q/k RMSNorm (+RoPE), head-major."""
    x = C.view(B, S, nq + nk + nv, 128)
    q = x[:, :, :nq].transpose(1, 2)
    k = x[:, :, nq:nq + nk].transpose(1, 2)
    v = x[:, :, nq + nk:].transpose(1, 2)
    if nq:
        q = dit_oracle.rms_norm(q, qw, eps)
    if nk:
        k = dit_oracle.rms_norm(k, kw, eps)
    if cos is not None:
        c, s_ = cos[None, None], sin[None, None]
        q = q * c + dit_oracle._rotate_half(q) * s_
        k = k * c + dit_oracle._rotate_half(k) * s_
    return q.contiguous(), k.contiguous(), v.contiguous()


@pytest.mark.parametrize("B,S,nq,nk,nv,K,rope", [
    (2, 300, 4, 2, 2, 256, True),      # ragged M (600 rows vs 192-row tiles), GQA q|k|v
    (1, 77, 2, 1, 1, 128, True),       # tiny-config layout: one 256-col tile mixes k and v heads
    (2, 250, 4, 0, 0, 192, False),     # cross-attention Q: q heads only, no RoPE
    (3, 65, 2, 2, 4, 64, True),        # one K-tile, B·S not a multiple of S-tiles
    (1, 125, 16, 8, 8, 2048, True),    # short song: split-K partials + standalone head_post
    (1, 3000, 16, 0, 0, 2048, False),  # cross-Q of the cond rows: half-chip grid → 192×128 one-head tiles
    (1, 2990, 8, 4, 4, 256, True),     # same tile choice with k / v heads, RoPE and a ragged last tile
    (2, 3000, 16, 8, 8, 256, True),    # the 240 s QKV grid: 256-row main round + 128-row tail round
])
def test_gemm_headpost_vs_oracle(gpu_device, B, S, nq, nk, nv, K, rope):
    ff = _ff()
    g = torch.Generator().manual_seed(B * 1000 + S + K)
    N = (nq + nk + nv) * 128
    A = torch.randn(B * S, K, generator=g).bfloat16()
    W = (torch.randn(N, K, generator=g) * 0.05).bfloat16()
    qw = (1 + 0.1 * torch.randn(128, generator=g)).bfloat16()
    kw = (1 + 0.1 * torch.randn(128, generator=g)).bfloat16()
    cos, sin = dit_oracle.rope_tables(S, 128, 1e6, torch.bfloat16) if rope else (None, None)
    if rope:
        cos, sin = cos[0].contiguous(), sin[0].contiguous()
    d = lambda t: None if t is None else t.to(gpu_device)
    Ad, Wd = d(A), d(W)
    qwd, kwd, cosd, sind = d(qw), d(kw), d(cos), d(sin)   # kept alive across the launch
    q = torch.zeros(B, nq, S, 128, dtype=torch.bfloat16, device=gpu_device)
    k = torch.zeros(B, nk, S, 128, dtype=torch.bfloat16, device=gpu_device)
    v = torch.zeros(B, nv, S, 128, dtype=torch.bfloat16, device=gpu_device)
    ff.check(ff.lib().acehip_gemm_headpost_bf16(
        ff.ptr(Ad), K, ff.ptr(Wd), K, B, S, nq, nk, nv, ff.ptr(qwd), ff.ptr(kwd), ff.ptr(cosd),
        ff.ptr(sind), 1e-6, ff.ptr(q) if nq else None, ff.ptr(k) if nk else None,
        ff.ptr(v) if nv else None, ff.stream_ptr()), "gemm_headpost")
    # same GEMM tile (variant 8) with the plain store epilogue → identical bf16(acc)
    C = torch.empty(B * S, N, dtype=torch.bfloat16, device=gpu_device)
    # (short songs take the split-K path: its plain-store twin is the production dispatch, -1)
    split = ((B * S + 127) // 128) * (N // 128) * 2 <= 256 and K // 64 >= 8
    ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(Ad), K, ff.ptr(Wd), K, ff.ptr(C), N, B * S, N, K, None, 0,
                                          -1 if split else 8, ff.stream_ptr()), "gemm")
    torch.cuda.synchronize()
    rq, rk, rv = _headpost_ref(C.cpu(), B, S, nq, nk, nv, qw, kw, cos, sin, 1e-6)
    for got, ref in ((q, rq), (k, rk), (v, rv)):
        if ref.numel() == 0:
            continue
        got = got.cpu()
        assert rel_l2(got.float(), ref.float()) < 2e-3
        assert (got != ref).float().mean().item() < 1e-3 + (0 if got is v else 5e-3)
    if nv:   # v heads are a pure scatter: bit-exact
        assert torch.equal(v.cpu(), rv)


@pytest.mark.parametrize("D", [2048, 256, 768])
@pytest.mark.parametrize("mod", [True, False])
def test_rmsnorm_variants_vs_oracle(gpu_device, D, mod):
    ff = _ff()
    g = torch.Generator().manual_seed(D + mod)
    M, rpb = 1001, 333                           # batch boundaries inside a 2- and 4-row wave
    nb = (M + rpb - 1) // rpb
    x = (torch.randn(M, D, generator=g) * 3).bfloat16()
    w = (1 + 0.1 * torch.randn(D, generator=g)).bfloat16()
    tab = (0.3 * torch.randn(nb, 6, D, generator=g)).bfloat16()   # mod rows 6·D apart like the DiT
    shift, scale = (tab[:, 0], tab[:, 1]) if mod else (None, None)
    ref = dit_oracle.rms_norm(x, w, 1e-6)
    if mod:
        b = torch.arange(M) // rpb
        ref = ref * (1 + scale[b]) + shift[b]
    xd, wd, td = x.to(gpu_device), w.to(gpu_device), tab.to(gpu_device)
    outs = []
    for r in (1, 2, 4, -2, -4):
        out = torch.empty(M, D, dtype=torch.bfloat16, device=gpu_device)
        ff.check(ff.lib().acehip_rmsnorm_bf16(
            ff.ptr(xd), ff.ptr(wd), ff.ptr(td[:, 0]) if mod else None, ff.ptr(td[:, 1]) if mod else None,
            6 * D, rpb, ff.ptr(out), M, D, 1e-6, r, ff.stream_ptr()), "rmsnorm")
        outs.append(out)
    torch.cuda.synchronize()
    # rows-per-wave changes scheduling, not arithmetic; the waves-per-row kernel (the
    # deferred split-K epilogue's norm) continues each lane's sum of squares across its waves
    # in element order, so it rounds identically too
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    got = outs[0].cpu()
    assert rel_l2(got.float(), ref.float()) < 2e-3
    assert (got != ref).float().mean().item() < 1e-3


@pytest.mark.parametrize("B,S,K", [(2, 3000, 2048), (2, 2500, 512), (7, 700, 256)])
def test_gemm_headpost_tail_split_bit_identical(gpu_device, monkeypatch, B, S, K):
    """The head-post GEMM as a tail split (whole rounds of 256-row tiles, the remaining rows as
    one round of 128-row tiles in the same launch, ACEHIP_GEMM_HPTAIL) gives the same bits as
    the 192-row grid: every output element accumulates the same K-tile MFMAs in the same order,
    and the tail grid's rows find their (b, s) through HeadPostArgs.m_off."""
    from conftest import set_knob
    ff = _ff()
    nq, nk, nv = 16, 8, 8
    N = (nq + nk + nv) * 128
    g = torch.Generator().manual_seed(B * S + K)
    A = torch.randn(B * S, K, generator=g).bfloat16().to(gpu_device)
    W = (torch.randn(N, K, generator=g) * 0.05).bfloat16().to(gpu_device)
    qw = (1 + 0.1 * torch.randn(128, generator=g)).bfloat16().to(gpu_device)
    kw = (1 + 0.1 * torch.randn(128, generator=g)).bfloat16().to(gpu_device)
    cos, sin = dit_oracle.rope_tables(S, 128, 1e6, torch.bfloat16)
    cos, sin = cos[0].contiguous().to(gpu_device), sin[0].contiguous().to(gpu_device)

    def run(tail):
        set_knob(monkeypatch, "ACEHIP_GEMM_HPTAIL", "1" if tail else "0")
        out = [torch.full((B, n, S, 128), float("nan"), dtype=torch.bfloat16, device=gpu_device)
               for n in (nq, nk, nv)]
        ff.check(ff.lib().acehip_gemm_headpost_bf16(
            ff.ptr(A), K, ff.ptr(W), K, B, S, nq, nk, nv, ff.ptr(qw), ff.ptr(kw), ff.ptr(cos), ff.ptr(sin), 1e-6,
            ff.ptr(out[0]), ff.ptr(out[1]), ff.ptr(out[2]), ff.stream_ptr()), "gemm_headpost")
        torch.cuda.synchronize()
        return out

    on, off = run(True), run(False)
    for a, b in zip(on, off):
        assert torch.isfinite(a.float()).all()
        assert torch.equal(a, b)
