"""Unit-level VAE parity (VERDICT r01 "weak" 2): every Oobleck conv kind at the decoder's and
encoder's real channel counts through the production kernels (acehip_vae_conv /
acehip_vae_resunit: weight packing, implicit-GEMM kernel selection, bf16 epilogues) against
fp32 torch.nn.functional.conv1d / conv_transpose1d on the same bf16-rounded operands
(acestep/models/mlx/vae_model.py:24-230 for the layer definitions and Snake1d).

Tolerance: the HIP path rounds the conv output to bf16 (and the residual sum and Snake each
once more); the fp32 reference does not round.  bf16 has 8 mantissa bits (relative
rounding ≤ 2^-9 ≈ 0.2 %), so a few roundings stay well below rel-L2 1e-2."""
import math

import pytest
import torch
import torch.nn.functional as F

from acehip import _ffi as ff
from conftest import set_knob

pytestmark = pytest.mark.gpu
TOL = 1e-2


def rel_l2(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


def snake(x, alpha, beta):
    # vae_model.py Snake1d with logscale parameters: x + 1/(e^β + 1e-9) · sin(e^α · x)²
    a, b = alpha.float().exp()[None, :], beta.float().exp()[None, :]
    return x + 1.0 / (b + 1e-9) * torch.sin(a * x) ** 2


def _bf(t):
    return t.to(torch.bfloat16)


def _run_conv(kind, x, w, bias, res, Cout, k, stride, dil, want_raw, alpha=None, beta=None):
    L = x.shape[0]
    L_out = L if kind == 0 else (L * stride if kind == 1 else L // stride)
    out = torch.empty(L_out, Cout, device=x.device, dtype=torch.bfloat16) if want_raw else None
    out_s = torch.empty(L_out, Cout, device=x.device, dtype=torch.bfloat16) if alpha is not None else None
    ff.check(ff.lib().acehip_vae_conv(kind, ff.ptr(x), L, x.shape[1], ff.ptr(w), ff.ptr(bias), ff.ptr(res), Cout,
                                      k, stride, dil, ff.ptr(out), ff.ptr(alpha), ff.ptr(beta), ff.ptr(out_s),
                                      ff.stream_ptr()), "vae_conv")
    return out, out_s


def _ref_conv(kind, x, w, bias, k, stride, dil):
    xi = x.float().t()[None]                                   # [1, Cin, L]
    b = bias.float() if bias is not None else None
    if kind == 0:
        y = F.conv1d(xi, w.float(), b, stride=1, padding=dil * (k - 1) // 2, dilation=dil)
    elif kind == 1:
        y = F.conv_transpose1d(xi, w.float(), b, stride=stride, padding=math.ceil(stride / 2))
    else:
        y = F.conv1d(xi, w.float(), b, stride=stride, padding=math.ceil(stride / 2))
    return y[0].t()                                            # [L_out, Cout]


# (kind, Cin, Cout, k, stride, dil, L, raw, res, snake): the decoder's ConvTranspose blocks
# (2048→1024 s10 … 128→128 s2), its k = 7 dilated convs (snake-only output: the halo-staged
# conv7 path), k = 1 convs with residual (C ≥ 256 residual tails), the encoder's strided convs
# and its k = 3 output conv
CASES = [
    (1, 2048, 1024, 20, 10, 1, 40, True, False, True),
    (1, 1024, 512, 12, 6, 1, 96, True, False, True),
    (1, 512, 256, 8, 4, 1, 300, True, False, True),
    (1, 256, 128, 8, 4, 1, 700, True, False, True),
    (1, 128, 128, 4, 2, 1, 1500, True, False, True),
    (0, 256, 256, 7, 1, 1, 1000, False, False, True),
    (0, 256, 256, 7, 1, 9, 1000, False, False, True),
    (0, 1024, 1024, 7, 1, 3, 300, False, False, True),
    (0, 128, 128, 7, 1, 3, 2000, False, False, True),
    (0, 512, 512, 1, 1, 1, 600, True, True, True),
    (0, 256, 256, 1, 1, 1, 900, False, True, True),
    (0, 256, 256, 7, 1, 9, 1000, True, True, False),
    (2, 128, 256, 4, 2, 1, 2000, True, False, True),
    (2, 1024, 2048, 20, 10, 1, 400, False, False, True),
    (0, 2048, 128, 3, 1, 1, 200, True, False, False),
]


@pytest.mark.parametrize("kind,Cin,Cout,k,stride,dil,L,raw,use_res,use_snake", CASES)
def test_vae_conv_unit(gpu_device, kind, Cin, Cout, k, stride, dil, L, raw, use_res, use_snake):
    g = torch.Generator(device=gpu_device).manual_seed(Cin * 7 + Cout + k + dil)
    x = _bf(torch.randn(L, Cin, device=gpu_device, generator=g))
    wshape = (Cin, Cout, k) if kind == 1 else (Cout, Cin, k)
    w = _bf(torch.randn(wshape, device=gpu_device, generator=g) / math.sqrt(Cin * k))
    bias = _bf(torch.randn(Cout, device=gpu_device, generator=g) * 0.1)
    L_out = L if kind == 0 else (L * stride if kind == 1 else L // stride)
    res = _bf(torch.randn(L_out, Cout, device=gpu_device, generator=g)) if use_res else None
    alpha = _bf(torch.randn(Cout, device=gpu_device, generator=g) * 0.3) if use_snake else None
    beta = _bf(torch.randn(Cout, device=gpu_device, generator=g) * 0.3) if use_snake else None
    out, out_s = _run_conv(kind, x, w, bias, res, Cout, k, stride, dil, raw, alpha, beta)
    torch.cuda.synchronize()
    y = _ref_conv(kind, x, w, bias, k, stride, dil)
    if use_res:
        y = res.float() + y
    if raw:
        assert rel_l2(out, y) < TOL, ("raw", rel_l2(out, y))
    if use_snake:
        ys = snake(y, alpha, beta)
        assert rel_l2(out_s, ys) < TOL, ("snake", rel_l2(out_s, ys))


@pytest.mark.parametrize("Cin,Cout,dil,L", [(256, 256, 1, 1000), (256, 256, 9, 1000), (512, 512, 3, 700),
                                          (1024, 1024, 3, 300), (1024, 1024, 9, 257), (512, 256, 1, 33)])
def test_vae_conv7_implicit_gemm(gpu_device, monkeypatch, Cin, Cout, dil, L):
    """ACEHIP_CONV7=2: the C ≥ 256 k = 7 convs as an implicit GEMM on the two-phase ping-pong
    tile (gemm.hip EPI_SNAKE; halo rows read from the zero rows around the activation) against
    the fp32 torch conv + Snake, and against the halo-staged conv7_kernel (both round the conv
    output to bf16 once before the Snake; only their fp32 accumulation orders differ).  L = 257
    and 33: partial last 256-row tiles; dil 9: the widest halo (27 rows each side)."""
    g = torch.Generator(device=gpu_device).manual_seed(Cin + Cout + dil + L)
    x = _bf(torch.randn(L, Cin, device=gpu_device, generator=g))
    w = _bf(torch.randn(Cout, Cin, 7, device=gpu_device, generator=g) / math.sqrt(Cin * 7))
    bias = _bf(torch.randn(Cout, device=gpu_device, generator=g) * 0.1)
    alpha = _bf(torch.randn(Cout, device=gpu_device, generator=g) * 0.3)
    beta = _bf(torch.randn(Cout, device=gpu_device, generator=g) * 0.3)
    set_knob(monkeypatch, "ACEHIP_CONV7", "2")
    _, gemm_s = _run_conv(0, x, w, bias, None, Cout, 7, 1, dil, False, alpha, beta)
    set_knob(monkeypatch, "ACEHIP_CONV7", "1")
    _, halo_s = _run_conv(0, x, w, bias, None, Cout, 7, 1, dil, False, alpha, beta)
    torch.cuda.synchronize()
    ys = snake(_ref_conv(0, x, w, bias, 7, 1, dil), alpha, beta)
    assert rel_l2(gemm_s, ys) < TOL, rel_l2(gemm_s, ys)
    assert rel_l2(gemm_s, halo_s) < 4e-3, rel_l2(gemm_s, halo_s)


@pytest.mark.parametrize("Cin,Cout,stride,L,raw,use_snake", [(2048, 1024, 10, 40, True, True), (1024, 512, 6, 96, True, True),
                                                            (512, 256, 4, 300, True, True), (512, 256, 4, 257, False, True),
                                                            (1024, 512, 6, 1, True, False), (256, 128, 4, 700, True, False),
                                                            (128, 128, 2, 1500, True, True), (128, 128, 2, 3, True, True)])
def test_vae_convt_implicit_gemm(gpu_device, monkeypatch, Cin, Cout, stride, L, raw, use_snake):
    """ACEHIP_CONVT=1: ConvTranspose1d (kernel 2s, stride s, padding ⌈s/2⌉) as the s phases'
    two-tap GEMMs side by side along N on the ping-pong tile (column n → channel n % Cout of
    phase n / Cout, output row m·s − pad + phase, rows outside [0, L·s) dropped; the C = 128
    blocks' Cout = 128 included) against torch's conv_transpose1d (+ Snake) and against the
    conv_gemm_kernel path (ACEHIP_CONVT=0).  L = 1: a single input row (every output row comes
    from the zero halo rows on one side)."""
    g = torch.Generator(device=gpu_device).manual_seed(Cin + Cout + stride + L)
    x = _bf(torch.randn(L, Cin, device=gpu_device, generator=g))
    w = _bf(torch.randn(Cin, Cout, 2 * stride, device=gpu_device, generator=g) / math.sqrt(Cin * 2))
    bias = _bf(torch.randn(Cout, device=gpu_device, generator=g) * 0.1)
    alpha = _bf(torch.randn(Cout, device=gpu_device, generator=g) * 0.3) if use_snake else None
    beta = _bf(torch.randn(Cout, device=gpu_device, generator=g) * 0.3) if use_snake else None
    set_knob(monkeypatch, "ACEHIP_CONVT", "1")
    out, out_s = _run_conv(1, x, w, bias, None, Cout, 2 * stride, stride, 1, raw, alpha, beta)
    set_knob(monkeypatch, "ACEHIP_CONVT", "0")
    out0, out_s0 = _run_conv(1, x, w, bias, None, Cout, 2 * stride, stride, 1, raw, alpha, beta)
    torch.cuda.synchronize()
    y = _ref_conv(1, x, w, bias, 2 * stride, stride, 1)
    if raw:
        assert rel_l2(out, y) < TOL, rel_l2(out, y)
        assert rel_l2(out, out0) < 4e-3, rel_l2(out, out0)
    if use_snake:
        ys = snake(y, alpha, beta)
        assert rel_l2(out_s, ys) < TOL, rel_l2(out_s, ys)
        assert rel_l2(out_s, out_s0) < 4e-3, rel_l2(out_s, out_s0)


@pytest.mark.parametrize("C,L,raw", [(256, 1000, True), (512, 600, False), (1024, 257, True)])
def test_vae_conv1_residual_gemm(gpu_device, monkeypatch, C, L, raw):
    """ACEHIP_CONVP=3: the C ≥ 256 residual units' k = 1 conv with its residual (x' = x +
    bf16(W2·y_s + b2), raw and/or snaked) as a plain GEMM on the ping-pong tile, vs torch fp32 and
    vs convp_kernel (ACEHIP_CONVP=2)."""
    g = torch.Generator(device=gpu_device).manual_seed(C + L)
    x = _bf(torch.randn(L, C, device=gpu_device, generator=g))
    w = _bf(torch.randn(C, C, 1, device=gpu_device, generator=g) / math.sqrt(C))
    bias = _bf(torch.randn(C, device=gpu_device, generator=g) * 0.1)
    res = _bf(torch.randn(L, C, device=gpu_device, generator=g))
    alpha = _bf(torch.randn(C, device=gpu_device, generator=g) * 0.3)
    beta = _bf(torch.randn(C, device=gpu_device, generator=g) * 0.3)
    set_knob(monkeypatch, "ACEHIP_CONVP", "3")
    out, out_s = _run_conv(0, x, w, bias, res, C, 1, 1, 1, raw, alpha, beta)
    set_knob(monkeypatch, "ACEHIP_CONVP", "2")
    out0, out_s0 = _run_conv(0, x, w, bias, res, C, 1, 1, 1, raw, alpha, beta)
    torch.cuda.synchronize()
    y = res.float() + _ref_conv(0, x, w, bias, 1, 1, 1)
    if raw:
        assert rel_l2(out, y) < TOL, rel_l2(out, y)
        assert rel_l2(out, out0) < 4e-3, rel_l2(out, out0)
    ys = snake(y, alpha, beta)
    assert rel_l2(out_s, ys) < TOL, rel_l2(out_s, ys)
    assert rel_l2(out_s, out_s0) < 4e-3, rel_l2(out_s, out_s0)


def _resunit(x, x_s, L, dil, w1, bb1, a2, be2, w2, bb2, an, ben, keep):
    C = x.shape[1]
    x_out = torch.empty(L, C, device=x.device, dtype=torch.bfloat16) if keep else None
    xs_out = torch.empty(L, C, device=x.device, dtype=torch.bfloat16)
    ff.check(ff.lib().acehip_vae_resunit(ff.ptr(x), ff.ptr(x_s), L, C, dil, ff.ptr(w1), ff.ptr(bb1), ff.ptr(a2),
                                         ff.ptr(be2), ff.ptr(w2), ff.ptr(bb2), ff.ptr(an), ff.ptr(ben),
                                         ff.ptr(x_out), ff.ptr(xs_out), ff.stream_ptr()), "vae_resunit")
    torch.cuda.synchronize()
    return x_out, xs_out


@pytest.mark.parametrize("ru", ["1", "2"])
@pytest.mark.parametrize("dil,L,keep", [(1, 3000, True), (3, 5000, False), (9, 70000, True), (9, 131, True),
                                        (9, 600000, True)])
def test_vae_resunit_c128(gpu_device, monkeypatch, dil, L, keep, ru):
    """The persistent C = 128 residual unit (ACEHIP_RU7=1: ru7_kernel, 128-row tiles; 2:
    ru8_kernel, 256-row tiles with DMA helper waves) vs the torch composition
    x + conv2(snake2(conv1(snake1(x)) + b1)) + b2 and snake_next of that; L = 70000 / 600000
    give ≥ 2 tiles per block (the cross-tile pipeline), L = 131 a ragged single partial tile.
    Both kernels accumulate in the same order, so ru8 must equal ru7 bit for bit."""
    set_knob(monkeypatch, "ACEHIP_RU7", ru)
    C = 128
    g = torch.Generator(device=gpu_device).manual_seed(dil * 100 + L)
    x = _bf(torch.randn(L, C, device=gpu_device, generator=g))
    a1, b1s = _bf(torch.randn(C, device=gpu_device, generator=g) * 0.3), _bf(torch.randn(C, device=gpu_device, generator=g) * 0.3)
    x_s = _bf(snake(x.float(), a1, b1s))
    w1 = _bf(torch.randn(C, C, 7, device=gpu_device, generator=g) / math.sqrt(C * 7))
    bb1 = _bf(torch.randn(C, device=gpu_device, generator=g) * 0.1)
    a2, be2 = _bf(torch.randn(C, device=gpu_device, generator=g) * 0.3), _bf(torch.randn(C, device=gpu_device, generator=g) * 0.3)
    w2 = _bf(torch.randn(C, C, 1, device=gpu_device, generator=g) / math.sqrt(C))
    bb2 = _bf(torch.randn(C, device=gpu_device, generator=g) * 0.1)
    an, ben = _bf(torch.randn(C, device=gpu_device, generator=g) * 0.3), _bf(torch.randn(C, device=gpu_device, generator=g) * 0.3)
    x_out, xs_out = _resunit(x, x_s, L, dil, w1, bb1, a2, be2, w2, bb2, an, ben, keep)
    if ru == "2":
        set_knob(monkeypatch, "ACEHIP_RU7", "1")
        x7, xs7 = _resunit(x, x_s, L, dil, w1, bb1, a2, be2, w2, bb2, an, ben, keep)
        assert torch.equal(xs_out, xs7), "ru8 out_s != ru7"
        if keep:
            assert torch.equal(x_out, x7), "ru8 x != ru7"
    y = F.conv1d(x_s.float().t()[None], w1.float(), bb1.float(), padding=3 * dil, dilation=dil)[0].t()
    y = snake(y, a2, be2)
    y = F.conv1d(y.t()[None], w2.float(), bb2.float())[0].t()
    xo = x.float() + y
    if keep:
        assert rel_l2(x_out, xo) < TOL, ("x_out", rel_l2(x_out, xo))
    xso = snake(xo, an, ben)
    assert rel_l2(xs_out, xso) < TOL, ("xs_out", rel_l2(xs_out, xso))
