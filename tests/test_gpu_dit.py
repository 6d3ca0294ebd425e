"""GPU parity: HIP kernels and the full DiT forward / sampler vs the oracle and
the reference's golden vectors.  Parity bar:
bf16 DiT output rel-L2 <= 2.5 % and cosine >= 0.999 vs the reference bf16
output on identical inputs; schedules bit-exact."""
import math

import pytest
import torch
import torch.nn.functional as F

from conftest import set_knob, cosine, golden_manifest, load_golden, rel_l2

from acehip.config import DiTConfig
from acehip.weights import synth_dit_weights
from oracle import dit_oracle, sampler_oracle

pytestmark = pytest.mark.gpu

TOL_REL, TOL_COS = 0.025, 0.999


def _lib():
    from acehip import _ffi
    return _ffi


@pytest.mark.parametrize("M,N,K", [(1000, 256, 384), (777, 2048, 2048), (6000, 128, 2048),
                                   (130, 4096, 6144)])
def test_gemm(gpu_device, M, N, K):
    ff = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(gpu_device, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * 0.02).to(gpu_device, torch.bfloat16)
    b = torch.randn(N, generator=g).to(gpu_device, torch.bfloat16)
    C = torch.empty(M, N, device=gpu_device, dtype=torch.bfloat16)
    ff.check(ff.lib().acehip_gemm_bf16(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(C), N, M, N, K, ff.ptr(b),
                                       ff.stream_ptr()))
    torch.cuda.synchronize()
    ref = A.float() @ W.float().t() + b.float()
    assert rel_l2(C.float().cpu(), ref.cpu()) < 5e-3
    # asymmetric check of the row/col mapping
    assert torch.allclose(C.float(), ref, atol=0.05, rtol=0.02)


EPI_STORE, EPI_GATED_RES, EPI_RES, EPI_SWIGLU = 0, 1, 2, 3


@pytest.mark.parametrize("variant", [0, 7, 8, 9, 13, 16, 17])
@pytest.mark.parametrize("M,N,K", [(300, 512, 64), (517, 256, 128), (200, 512, 192), (777, 768, 640)])
def test_gemm_variants(gpu_device, variant, M, N, K):
    """Every production tile variant, odd K-tile counts (ring prologue/tail) and ragged M,
    plain store + SwiGLU epilogue (gate/up interleaved in 32-row panels)."""
    _gemm_variant_check(gpu_device, variant, M, N, K)


@pytest.mark.parametrize("M,N,K", [(517, 256, 128), (777, 768, 640)])
def test_gemm_four_wave_without_helpers(gpu_device, monkeypatch, M, N, K):
    """The half-chip four-wave tile without its LDS-DMA helper waves (ACEHIP_GEMM_HELPERS=0, A/B arm)."""
    set_knob(monkeypatch, "ACEHIP_GEMM_HELPERS", "0")
    _gemm_variant_check(gpu_device, 13, M, N, K)


def _gemm_variant_check(gpu_device, variant, M, N, K):
    ff = _lib()
    if variant in (7, 8, 9) and N % 256:
        pytest.skip("variant needs N % 256 == 0")
    g = torch.Generator(device="cpu").manual_seed(M * 3 + N + K + variant)
    A = torch.randn(M, K, generator=g).to(gpu_device, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * 0.05).to(gpu_device, torch.bfloat16)
    C = torch.empty(M, N, device=gpu_device, dtype=torch.bfloat16)
    ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(C), N, M, N, K, None, EPI_STORE,
                                          variant, ff.stream_ptr()))
    torch.cuda.synchronize()
    ref = A.float() @ W.float().t()
    assert rel_l2(C.float().cpu(), ref.cpu()) < 5e-3
    assert torch.allclose(C.float(), ref, atol=0.05, rtol=0.02)
    # SwiGLU: packed rows = per 64-row panel [32 gate ; 32 up] -> out[:, N/2]
    Cs = torch.empty(M, N // 2, device=gpu_device, dtype=torch.bfloat16)
    ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(Cs), N // 2, M, N, K, None,
                                          EPI_SWIGLU, variant, ff.stream_ptr()))
    torch.cuda.synchronize()
    y = ref.bfloat16().float().view(M, N // 64, 2, 32)
    gate, up = y[:, :, 0, :].reshape(M, N // 2), y[:, :, 1, :].reshape(M, N // 2)
    refs = torch.nn.functional.silu(gate).bfloat16().float() * up
    assert rel_l2(Cs.float().cpu(), refs.cpu()) < 1e-2


@pytest.mark.parametrize("cus,window", [(16, -1), (18, -1), (20, -1)])
@pytest.mark.parametrize("pw", ["0", "7"])
def test_attention_tail_split(gpu_device, monkeypatch, cus, window, pw):
    """Tail balancing with 2-, 3- and 4-way KV splits (24 units; CU count 16/18/20 → tail 8/6/4 →
    nsplit 2/3/4; overridden so small
    shapes take the split path): merged partials must match the fp32 reference."""
    set_knob(monkeypatch, "ACEHIP_ATTN_CUS", str(cus))
    set_knob(monkeypatch, "ACEHIP_ATTN_PW", pw)
    ff = _lib()
    B, H, KV, Sq, Sk = 2, 4, 2, 700, 1600       # 6 q-blocks x 2 KV x 2 = 24 units, 25 KV tiles
    g = torch.Generator(device="cpu").manual_seed(cus * 3 + window)
    q = torch.randn(B, H, Sq, 128, generator=g).to(gpu_device, torch.bfloat16)
    k = torch.randn(B, KV, Sk, 128, generator=g).to(gpu_device, torch.bfloat16)
    v = torch.randn(B, KV, Sk, 128, generator=g).to(gpu_device, torch.bfloat16)
    outs = []
    for _ in range(3):                          # later launches check the counters self-reset
        o = torch.empty(B, Sq, H * 128, device=gpu_device, dtype=torch.bfloat16)
        ff.check(ff.lib().acehip_attention_bf16(ff.ptr(q), ff.ptr(k), ff.ptr(v), ff.ptr(o), B, H, KV, Sq, Sk,
                                                window, 1 / math.sqrt(128), ff.stream_ptr()))
        torch.cuda.synchronize()
        ref = _attn_ref(q, k, v, window).transpose(1, 2).reshape(B, Sq, H * 128)
        assert rel_l2(o.float().cpu(), ref.float().cpu()) < 1e-2
        outs.append(o)
    # the parts are merged in part order whichever finishes last: bit-reproducible
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("B,H,KV,Sq,Sk,cus", [(1, 16, 8, 125, 641, 0), (1, 16, 8, 125, 125, 0),
                                               (2, 16, 8, 125, 641, 0), (1, 16, 8, 1, 641, 0),
                                               (1, 2, 1, 33, 65, 0), (3, 4, 2, 77, 1000, 0),
                                               (1, 16, 16, 200, 2000, 0), (1, 16, 8, 125, 641, 100),
                                               (1, 4, 2, 31, 3000, 64), (1, 2, 1, 40, 1, 0)])
def test_attention_small(gpu_device, monkeypatch, B, H, KV, Sq, Sk, cus):
    """attn_small_kernel (few-unit unmasked full / cross attention, the turbo 10 s song): one head
    × 32 query rows per workgroup, KV tiles interleaved over four waves, their partials folded in
    LDS, and the unit's KV parts (ACEHIP_ATTN_SMALL=1: about one tile per wave, 1 to 16 parts)
    folded through the workspace in part order.  Against the fp32 reference; bit-reproducible
    over launches (the tickets self-reset); parts vs no parts (=2) within rounding."""
    if cus:
        set_knob(monkeypatch, "ACEHIP_ATTN_CUS", str(cus))
    ff = _lib()
    g = torch.Generator(device="cpu").manual_seed(Sq * 7 + Sk + B)
    q = torch.randn(B, H, Sq, 128, generator=g).to(gpu_device, torch.bfloat16)
    k = torch.randn(B, KV, Sk, 128, generator=g).to(gpu_device, torch.bfloat16)
    v = torch.randn(B, KV, Sk, 128, generator=g).to(gpu_device, torch.bfloat16)
    ref = _attn_ref(q, k, v, -1).transpose(1, 2).reshape(B, Sq, H * 128).float().cpu()
    outs = {}
    for mode in ("1", "2"):
        set_knob(monkeypatch, "ACEHIP_ATTN_SMALL", mode)
        runs = []
        for _ in range(3):
            o = torch.full((B, Sq, H * 128), float("nan"), device=gpu_device, dtype=torch.bfloat16)
            ff.check(ff.lib().acehip_attention_bf16(ff.ptr(q), ff.ptr(k), ff.ptr(v), ff.ptr(o), B, H, KV, Sq, Sk,
                                                    -1, 1 / math.sqrt(128), ff.stream_ptr()))
            torch.cuda.synchronize()
            runs.append(o)
        assert torch.equal(runs[0], runs[1]) and torch.equal(runs[0], runs[2])
        assert rel_l2(runs[0].float().cpu(), ref) < 1e-2
        outs[mode] = runs[0].float().cpu()
    assert rel_l2(outs["1"], outs["2"]) < 1e-2


@pytest.mark.parametrize("cus,B,H,KV,S,window", [(16, 2, 4, 2, 1000, 128), (37, 2, 4, 2, 1000, 128),
                                                  (100, 1, 16, 8, 777, 64), (7, 1, 2, 1, 450, 200),
                                                  (0, 2, 16, 8, 3000, 128), (0, 4, 16, 8, 3000, 128)])
def test_attention_band_persistent(gpu_device, monkeypatch, cus, B, H, KV, S, window):
    """Band layers with more units than CUs run attn_pw_kernel persistently (one workgroup per
    CU walking units blockIdx + k·grid as one KV-tile stream: the next unit's tiles staged during
    the current unit's last two, its Q loaded behind the last tile's barrier).  ACEHIP_ATTN_CUS
    shrinks the grid so small shapes walk 2..10 units per workgroup (odd tile counts flip the
    ring parity between units; ragged S leaves a partial last tile); cus = 0 keeps the real
    CU count (the 240 s / 2- and 3-round shapes).  Bit-identical to one workgroup per unit."""
    if cus:
        set_knob(monkeypatch, "ACEHIP_ATTN_CUS", str(cus))
    set_knob(monkeypatch, "ACEHIP_ATTN_PW", "2")
    ff = _lib()
    g = torch.Generator(device="cpu").manual_seed(S + cus)
    q = torch.randn(B, H, S, 128, generator=g).to(gpu_device, torch.bfloat16)
    k = torch.randn(B, KV, S, 128, generator=g).to(gpu_device, torch.bfloat16)
    v = torch.randn(B, KV, S, 128, generator=g).to(gpu_device, torch.bfloat16)
    outs = {}
    for pers in ("1", "0"):
        set_knob(monkeypatch, "ACEHIP_ATTN_PERSIST", pers)
        o = torch.full((B, S, H * 128), float("nan"), device=gpu_device, dtype=torch.bfloat16)
        ff.check(ff.lib().acehip_attention_bf16(ff.ptr(q), ff.ptr(k), ff.ptr(v), ff.ptr(o), B, H, KV, S, S,
                                                window, 1 / math.sqrt(128), ff.stream_ptr()))
        torch.cuda.synchronize()
        outs[pers] = o
    ref = _attn_ref(q, k, v, window).transpose(1, 2).reshape(B, S, H * 128)
    assert rel_l2(outs["1"].float().cpu(), ref.cpu()) < 1e-2
    assert torch.equal(outs["1"], outs["0"])


def _attn_ref(q, k, v, window):
    Sq, Sk = q.shape[2], k.shape[2]
    rep = q.shape[1] // k.shape[1]
    k = k.float().repeat_interleave(rep, 1)
    v = v.float().repeat_interleave(rep, 1)
    s = (q.float() @ k.transpose(2, 3)) / math.sqrt(128)
    i = torch.arange(Sq, device=q.device)[:, None]
    j = torch.arange(Sk, device=q.device)[None, :]
    if window >= 0:
        s = s.masked_fill((i - j).abs() > window, float("-inf"))
    elif window == -2:                                  # causal (Qwen3 text encoder)
        s = s.masked_fill(j > i, float("-inf"))
    return torch.softmax(s, -1) @ v


@pytest.mark.parametrize("B,H,KV,Sq,Sk,window", [(2, 4, 2, 300, 300, -1), (2, 4, 2, 300, 300, 8),
                                                  (1, 16, 8, 1000, 1000, 128), (2, 4, 2, 257, 641, -1),
                                                  (1, 2, 1, 50, 20, -1), (1, 2, 1, 3000, 3000, 128),
                                                  # DiT shapes at 240 s: 384 units on 256 CUs → tail split (full),
                                                  # GQA pair split into two 4-wave workgroups (band, cross)
                                                  (2, 16, 8, 3000, 3000, -1), (2, 16, 8, 3000, 3000, 128),
                                                  (2, 16, 8, 3000, 641, -1),
                                                  # 10 s song: 8 units → every unit KV-split
                                                  (1, 16, 8, 125, 641, -1), (1, 16, 8, 125, 125, 128),
                                                  # causal: text encoder (128 tokens), ragged, nrep 1
                                                  (2, 16, 8, 128, 128, -2), (1, 16, 8, 77, 77, -2),
                                                  (3, 4, 2, 300, 300, -2), (1, 2, 2, 257, 257, -2)])
@pytest.mark.parametrize("pw", ["0", "7"])
def test_attention(gpu_device, monkeypatch, B, H, KV, Sq, Sk, window, pw):
    """pw: ACEHIP_ATTN_PW — "0" every layer kind on attn_fwd_kernel, "7" the GQA-pair unmasked
    kinds (full / band / cross) on the 64-row-per-wave attn_pw_kernel (production: band only)."""
    set_knob(monkeypatch, "ACEHIP_ATTN_PW", pw)
    ff = _lib()
    g = torch.Generator(device="cpu").manual_seed(Sq * 7 + Sk)
    q = torch.randn(B, H, Sq, 128, generator=g).to(gpu_device, torch.bfloat16)
    k = torch.randn(B, KV, Sk, 128, generator=g).to(gpu_device, torch.bfloat16)
    v = torch.randn(B, KV, Sk, 128, generator=g).to(gpu_device, torch.bfloat16)
    o = torch.empty(B, Sq, H * 128, device=gpu_device, dtype=torch.bfloat16)
    ff.check(ff.lib().acehip_attention_bf16(ff.ptr(q), ff.ptr(k), ff.ptr(v), ff.ptr(o), B, H, KV, Sq, Sk,
                                            window, 1 / math.sqrt(128), ff.stream_ptr()))
    torch.cuda.synchronize()
    ref = _attn_ref(q, k, v, window).transpose(1, 2).reshape(B, Sq, H * 128)
    assert rel_l2(o.float().cpu(), ref.cpu()) < 1e-2


def _runtime(cfg, W, gpu_device, max_S=64, max_Bc=2, max_Lenc=32):
    from acehip.dit import DiTRuntime
    rt = DiTRuntime(cfg, gpu_device.index or 0, max_S=max_S, max_Bc=max_Bc, max_Lenc=max_Lenc)
    rt.load({k: v.to(gpu_device, torch.bfloat16) for k, v in W.items()})
    return rt


@pytest.mark.parametrize("name", ["tiny_bfloat16", "tiny_odd_bfloat16", "full2_bfloat16",
                                  # full width, T = 641 (S = 321 > 2W+1: the ±128 band is pinned)
                                  "full2_long_bfloat16"])
def test_dit_forward_vs_reference_golden(gpu_device, name):
    meta = golden_manifest()["forward"][name]
    cfg = DiTConfig(**meta["cfg"])
    g = load_golden("dit_fwd_" + name)
    W = synth_dit_weights(cfg, seed=meta["seed"], mode="parity")
    rt = _runtime(cfg, W, gpu_device, max_S=max(64, (meta["T"] + 1) // 2), max_Lenc=max(32, meta["Lenc"]))
    rt.set_condition(g["enc"].to(gpu_device))
    out = rt.forward(g["xt"].to(gpu_device).contiguous(), g["ctx"].to(gpu_device).contiguous(),
                     g["t"].float().to(gpu_device), g["t_r"].float().to(gpu_device))
    torch.cuda.synchronize()
    out = out.float().cpu()
    ref = g["vt"].float()
    assert rel_l2(out, ref) <= TOL_REL, rel_l2(out, ref)
    assert cosine(out, ref) >= TOL_COS
    if torch.equal(g["t"], g["t"][:1].expand(2)) and torch.equal(g["t_r"], g["t_r"][:1].expand(2)):
        # one timestep for both rows (the sampler's t_curr·ones(Bc), base:1929-1941): a broadcast
        # t (t_stride 0) and the schedule path (set_timesteps + forward_step) vs the same golden
        xd, cd = g["xt"].to(gpu_device).contiguous(), g["ctx"].to(gpu_device).contiguous()
        bc = rt.forward(xd, cd, g["t"][:1].float().to(gpu_device), g["t_r"][:1].float().to(gpu_device)).float().cpu()
        rt.set_timesteps(torch.tensor([1.0, float(g["t"][0])], device=gpu_device),
                         torch.tensor([1.0, float(g["t_r"][0])], device=gpu_device))
        st = rt.forward_step(xd, cd, 1).float().cpu()
        torch.cuda.synchronize()
        for o in (bc, st):
            assert rel_l2(o, ref) <= TOL_REL and cosine(o, ref) >= TOL_COS, rel_l2(o, ref)
        assert torch.equal(bc, st)
    rt.close()


@pytest.mark.parametrize("name", ["full2_bfloat16", "full2_long_bfloat16"])
def test_profile_events_do_not_change_results(gpu_device, name):
    """acehip_dit_profile: the SwiGLU GEMM's timing events ride on its launches
    (hipExtLaunchKernel start / stop, gemm_ext_events) and the other kinds are bracketed by
    event records — every kind reports one launch per layer with a positive time, and the
    forward is bit-identical with and without profiling (small-M whole-K and larger-M paths)."""
    meta = golden_manifest()["forward"][name]
    cfg = DiTConfig(**meta["cfg"])
    g = load_golden("dit_fwd_" + name)
    W = synth_dit_weights(cfg, seed=meta["seed"], mode="parity")
    rt = _runtime(cfg, W, gpu_device, max_S=max(64, (meta["T"] + 1) // 2), max_Lenc=max(32, meta["Lenc"]))
    rt.set_condition(g["enc"].to(gpu_device))
    args = (g["xt"].to(gpu_device).contiguous(), g["ctx"].to(gpu_device).contiguous(),
            g["t"].float().to(gpu_device), g["t_r"].float().to(gpu_device))
    plain = rt.forward(*args).clone()
    for kinds in (["gemm_swiglu"], None):
        rt.profile(True, kinds=kinds)
        prof = rt.forward(*args).clone()
        torch.cuda.synchronize()
        stats = rt.profile_read()
        rt.profile(False)
        assert torch.equal(plain, prof)
        n, ms = stats["gemm_swiglu"]
        assert n == cfg.num_hidden_layers and ms > 0, stats
        if kinds is None:
            assert stats["gemm_qkv"][0] == cfg.num_hidden_layers and stats["gemm_qkv"][1] > 0
    rt.close()


def test_dit_forward_cfg_rows_and_long_sequence(gpu_device):
    """Bx < Bc (CFG reads xt row b % Bx), odd T, band + full layers at S > 2·window,
    Lenc not a multiple of 64 — vs the bf16 CPU oracle."""
    cfg = DiTConfig.tiny(layers=4, window=16)
    W = synth_dit_weights(cfg, seed=5, mode="parity")
    g = torch.Generator().manual_seed(3)
    B, T, Lenc = 1, 401, 77
    xt = torch.randn(B, T, 64, generator=g).bfloat16()
    ctx = torch.randn(B, T, 128, generator=g).bfloat16()
    enc = torch.randn(2 * B, Lenc, cfg.hidden_size, generator=g).bfloat16()
    t = torch.tensor([0.8], dtype=torch.bfloat16)
    Wb = {k: v.bfloat16() for k, v in W.items()}
    with torch.no_grad():
        ref = dit_oracle.dit_forward(Wb, cfg, torch.cat([xt, xt]), t.expand(2), t.expand(2), enc,
                                     torch.cat([ctx, ctx]))
    rt = _runtime(cfg, W, gpu_device, max_S=256, max_Lenc=128)
    rt.set_condition(enc.to(gpu_device))
    out = rt.forward(xt.to(gpu_device), ctx.to(gpu_device), t.float().to(gpu_device)).float().cpu()
    assert rel_l2(out, ref.float()) <= TOL_REL
    assert cosine(out, ref.float()) >= TOL_COS
    rt.close()


@pytest.mark.parametrize("name", ["base_s8_sh3", "base_s27_sh3", "base_s60_sh3",
                                  "base_s10_sh1_interval"])
def test_apg_euler_kernel_replay(gpu_device, name):
    """Drive the fused HIP APG+Euler kernel with the reference's recorded
    decoder outputs; every step's x must match the reference's."""
    from acehip.dit import apg_euler_, base_schedule
    meta = golden_manifest()["sampler"][name]
    kw = meta["kwargs"]
    gd = load_golden("sampler_" + name)
    B = meta["B"]
    t = base_schedule(kw["infer_steps"], kw.get("shift", 1.0), gpu_device, torch.bfloat16)
    dts = (t[:-1] - t[1:]).float().tolist()
    s, e = kw.get("cfg_interval_start", 0.0), kw.get("cfg_interval_end", 1.0)
    on = ((t[:-1] >= s) & (t[:-1] <= e)).tolist()
    xt = gd["x_0"][:B].to(gpu_device).contiguous()
    ra = torch.zeros_like(xt)
    first = True
    worst = 0.0
    for i in range(meta["n_calls"]):
        ref_x = gd[f"x_{i}"][:B].float()
        d = (xt.float().cpu() - ref_x).abs().max().item()
        worst = max(worst, d)
        vt = gd[f"vt_{i}"].to(gpu_device).contiguous()
        apply = 1 if on[i] else 0
        apg_euler_(vt, xt, ra, kw["diffusion_guidance_sale"], dts[i], apply, first and apply == 1)
        if apply:
            first = False
    torch.cuda.synchronize()
    out = xt.float().cpu()
    ref = gd["target_latents"].float()
    # reductions run in a different order than torch's (fp32/fp64): allow a
    # few bf16 ulps of drift, far inside the forward tolerance
    assert rel_l2(out, ref) < 5e-3, (rel_l2(out, ref), worst)


@pytest.mark.parametrize("T,dtype", [(6000, torch.bfloat16), (1001, torch.bfloat16), (6000, torch.float32),
                                     (1001, torch.float32)])
def test_apg_euler_multichunk(gpu_device, T, dtype):
    """The APG step's per-(song, channel) norms over T are reduced across 256-row chunks in
    three launches (csrc/sampler.hip): at production length (T = 6000: 24 chunks) and at a
    ragged length (T = 1001: 4 chunks, the last one 233 rows), B = 2, CFG toggling on/off
    and the first-step momentum reset, every step compared with the oracle's apg
    (apg_guidance.py:16-56) + Euler (base:1975-1979) started from the device's own state
    (xt, momentum buffer) so each step is checked on identical inputs."""
    from acehip.dit import apg_euler_
    B, C, guidance = 2, 64, 7.0
    g = torch.Generator().manual_seed(T)
    xt = torch.randn(B, T, C, generator=g).to(dtype)
    ra = torch.zeros(B, T, C, dtype=dtype)
    xd, rd = xt.to(gpu_device).contiguous(), ra.to(gpu_device).contiguous()
    plan = [(1, 1), (1, 0), (0, 0), (1, 0), (1, 0)]        # (apply_cfg, first_step)
    for step, (apply, first) in enumerate(plan):
        vt = (torch.randn(2 * B, T, C, generator=g) * (1.0 + step)).to(dtype)
        dt = float(torch.tensor(0.0371 * (step + 1), dtype=dtype))
        x0, r0 = xd.cpu(), rd.cpu()
        apg_euler_(vt.to(gpu_device).contiguous(), xd, rd, guidance, dt, apply, first)
        torch.cuda.synchronize()
        cond, uncond = vt.chunk(2)
        if apply:
            mom = sampler_oracle.Momentum()
            mom.running_average = 0 if first else r0
            v = sampler_oracle.apg(cond, uncond, guidance, mom, dims=(1,))
            ref_r = mom.running_average
        else:
            v, ref_r = cond, r0
        ref_x = x0 - v * torch.tensor(dt, dtype=dtype)
        got_x, got_r = xd.cpu(), rd.cpu()
        # the momentum update is elementwise: exact; the norms' reduction order differs from
        # torch's, which can move a clip scale by an ulp -> a bf16 ulp of drift in a few elements
        if dtype == torch.bfloat16:      # every op rounded to bf16: exact
            assert torch.equal(got_r, ref_r.to(dtype)), step
        else:                            # fp32: hipcc may contract the update into an FMA
            assert rel_l2(got_r, ref_r) < 1e-6, step
        if dtype == torch.bfloat16:
            # every op of the chain rounded as torch rounds it, including the clip scale
            # 2.5 / ‖diff‖ = bf16(bf16(1/‖diff‖)·2.5) (torch's __rtruediv__).  What remains is
            # the order of the fp64 projection sum Σ v0·v1 over T: it can move orth across a
            # float / bf16 rounding tie in an isolated element (measured: 1 of 768,000 at
            # T = 6000) — allowed up to 1e-5 of the elements, every other element bit-exact
            mism = int((got_x != ref_x).sum())
            assert mism <= max(1, got_x.numel() // 100_000), (step, mism, rel_l2(got_x.float(), ref_x.float()))
            assert (got_x.float() - ref_x.float()).abs().max() <= ref_x.float().abs().max() * 2 ** -7
        else:
            r = rel_l2(got_x.float(), ref_x.float())
            assert r < 1e-5, (step, r)


def test_schedule_bit_exact_on_device(gpu_device):
    from acehip.dit import base_schedule
    for steps, shift in ((8, 3.0), (27, 3.0), (60, 3.0), (10, 1.0)):
        dev = base_schedule(steps, shift, gpu_device, torch.bfloat16).cpu()
        cpu = sampler_oracle.base_schedule(steps, shift, torch.bfloat16)
        assert torch.equal(dev.view(torch.int16), cpu.view(torch.int16)), (steps, shift)


@pytest.mark.parametrize("i", range(4))
def test_adg_kernel_vs_reference(gpu_device, i):
    """Fused HIP ADG (out_mode=1: the guided velocity) against the reference's
    adg_forward outputs.  Rows the reference leaves finite must agree to bf16
    rounding (fp64 acos/sin/cos and wave-order sums may move a value by one
    ulp); the near-parallel row whose fp64 cos rounds above 1 is NaN in the
    reference and order-dependent here, so it is excluded."""
    from acehip.dit import adg_euler_
    g = load_golden("adg_direct")
    guidance = golden_manifest()["adg"]["direct"]["guidance"]
    x, c, u = g[f"x_{i}"], g[f"cond_{i}"], g[f"uncond_{i}"]
    vt = torch.cat([c, u]).to(gpu_device).contiguous()
    v = x.to(gpu_device).contiguous()
    adg_euler_(vt, v, guidance, float(g[f"sigma_{i}"].float()), 0.0, out_mode=1)
    torch.cuda.synchronize()
    out, ref = v.float().cpu(), g[f"out_{i}"].float()
    rows_ok = ~ref.isnan().any(-1)
    rows_ok[:, 3] = False
    o, r = out[rows_ok], ref[rows_ok]
    assert torch.isfinite(o).all()
    ulp = (r.abs() * 2.0 ** -7).clamp_min(1e-30)
    assert ((o - r).abs() <= ulp + 1e-6).float().mean() >= 0.999
    assert rel_l2(o, r) < 1e-3


def test_adg_sampler_replay(gpu_device):
    """A whole 8-step base generate_audio with use_adg=True, replayed with the
    reference's recorded decoder outputs through the fused ADG+Euler kernel."""
    from acehip.dit import adg_euler_, base_schedule
    meta = golden_manifest()["sampler"]["base_s8_adg"]
    kw = meta["kwargs"]
    gd = load_golden("sampler_base_s8_adg")
    B = meta["B"]
    t = base_schedule(kw["infer_steps"], kw["shift"], gpu_device, torch.bfloat16)
    dts = (t[:-1] - t[1:]).float().tolist()
    th = t.float().tolist()
    xt = gd["x_0"][:B].to(gpu_device).contiguous()
    for i in range(meta["n_calls"]):
        assert rel_l2(xt.float().cpu(), gd[f"x_{i}"][:B].float()) < 5e-3, i
        vt = gd[f"vt_{i}"].to(gpu_device).contiguous()
        adg_euler_(vt, xt, kw["diffusion_guidance_sale"], th[i], dts[i])
    torch.cuda.synchronize()
    assert rel_l2(xt.float().cpu(), gd["target_latents"].float()) < 5e-3


def test_generate_audio_adg_runs(gpu_device):
    """generate_audio(use_adg=True) end to end on the HIP path (ODE and SDE)."""
    from acehip.dit import AceStepDiTBackend
    cfg = DiTConfig.tiny(layers=2, window=8)
    W = synth_dit_weights(cfg, seed=9, mode="parity")
    null = torch.randn(1, 1, cfg.hidden_size, generator=torch.Generator().manual_seed(1))
    rt = _runtime(cfg, W, gpu_device, max_S=64, max_Bc=2, max_Lenc=32)
    be = AceStepDiTBackend(rt, null, is_turbo=False)
    g = torch.Generator().manual_seed(3)
    enc = torch.randn(1, 16, cfg.hidden_size, generator=g).bfloat16().to(gpu_device)
    ctx = torch.randn(1, 40, 128, generator=g).bfloat16().to(gpu_device)
    for method in ("ode", "sde"):
        res = be.generate_audio(encoder_hidden_states=enc, context_latents=ctx, infer_steps=4,
                                diffusion_guidance_sale=5.0, shift=3.0, seed=0, use_adg=True,
                                infer_method=method)
        torch.cuda.synchronize()
        assert res["target_latents"].shape == (1, 40, 64)
        assert torch.isfinite(res["target_latents"].float()).all()
    rt.close()


def test_generate_audio_per_step_parity(gpu_device):
    """Full base/sft generate_audio (CFG 7 + APG, shift 3) on the HIP path; at
    every step the HIP DiT output is checked against the CPU oracle fed the
    HIP path's own x_t (per-step parity)."""
    from acehip.dit import AceStepDiTBackend, DiTRuntime
    cfg = DiTConfig.tiny(layers=2, window=8)
    W = synth_dit_weights(cfg, seed=9, mode="parity")
    null = torch.randn(1, 1, cfg.hidden_size, generator=torch.Generator().manual_seed(1))
    rt = _runtime(cfg, W, gpu_device, max_S=64, max_Bc=4, max_Lenc=32)
    be = AceStepDiTBackend(rt, null, is_turbo=False)
    g = torch.Generator().manual_seed(0)
    B, T, Lenc = 2, 60, 24
    enc = torch.randn(B, Lenc, cfg.hidden_size, generator=g).bfloat16()
    ctx = torch.randn(B, T, 128, generator=g).bfloat16()
    seen = []
    orig = rt.forward

    orig_step = rt.forward_step

    def spy(xt, c, t, t_r=None, out=None):
        vt = orig(xt, c, t, t_r, out)
        seen.append((xt.clone(), t.clone(), vt.clone()))
        return vt

    def spy_step(xt, c, step, out=None):      # the production path (acehip_dit_forward_step)
        vt = orig_step(xt, c, step, out)
        seen.append((xt.clone(), rt._ts[0][step:step + 1].clone(), vt.clone()))
        return vt
    rt.forward = spy
    rt.forward_step = spy_step
    res = be.generate_audio(encoder_hidden_states=enc.to(gpu_device), context_latents=ctx.to(gpu_device),
                            infer_steps=4, diffusion_guidance_sale=7.0, shift=3.0, seed=[0, 1])
    torch.cuda.synchronize()
    assert res["target_latents"].shape == (B, T, 64)
    assert set(res["time_costs"]) >= {"encoder_time_cost", "diffusion_time_cost",
                                      "diffusion_per_step_time_cost", "total_time_cost"}
    Wb = {k: v.bfloat16() for k, v in W.items()}
    enc2 = torch.cat([enc, null.bfloat16().expand_as(enc)])
    kv = dit_oracle.cross_kv(Wb, cfg, enc2)
    assert len(seen) == 4
    for xt, t, vt in seen:
        x2 = torch.cat([xt, xt]).cpu()
        tv = t.cpu().bfloat16().expand(2 * B)
        with torch.no_grad():
            ref = dit_oracle.dit_forward(Wb, cfg, x2, tv, tv, enc2, torch.cat([ctx, ctx]), kv_cache=kv)
        assert rel_l2(vt.float().cpu(), ref.float()) <= TOL_REL
        assert cosine(vt.float().cpu(), ref.float()) >= TOL_COS
    rt.close()


def test_turbo_generate_audio_runs(gpu_device):
    from acehip.dit import AceStepDiTBackend
    cfg = DiTConfig.tiny(layers=2, window=8)
    W = synth_dit_weights(cfg, seed=4, mode="parity")
    null = torch.zeros(1, 1, cfg.hidden_size)
    rt = _runtime(cfg, W, gpu_device, max_S=64, max_Bc=2, max_Lenc=32)
    be = AceStepDiTBackend(rt, null, is_turbo=True)
    g = torch.Generator().manual_seed(0)
    enc = torch.randn(1, 16, cfg.hidden_size, generator=g).bfloat16().to(gpu_device)
    ctx = torch.randn(1, 40, 128, generator=g).bfloat16().to(gpu_device)
    res = be.generate_audio(encoder_hidden_states=enc, context_latents=ctx, shift=3.0, seed=0)
    x = res["target_latents"]
    assert x.shape == (1, 40, 64) and torch.isfinite(x.float()).all()
    rt.close()


def test_uniform_null_rows_closed_form(gpu_device):
    """CFG null rows (null_condition_emb repeated, base:1907): the closed-form cross-attention
    (acehip_dit_set_uniform_rows) equals the full computation of those rows."""
    from acehip.dit import DiTRuntime
    cfg = DiTConfig.tiny(layers=4, window=8)
    W = synth_dit_weights(cfg, seed=3, mode="parity")
    rt = DiTRuntime(cfg, 0, max_S=64, max_Bc=4, max_Lenc=40)
    rt.load({k: v.to(gpu_device, torch.bfloat16) for k, v in W.items()})
    g = torch.Generator().manual_seed(5)
    B, T, Le = 2, 100, 37
    xt = torch.randn(B, T, 64, generator=g).bfloat16().to(gpu_device)
    ctx = torch.randn(B, T, 128, generator=g).bfloat16().to(gpu_device)
    enc = torch.randn(B, Le, cfg.hidden_size, generator=g).bfloat16()
    null = torch.randn(1, 1, cfg.hidden_size, generator=g).bfloat16()
    encc = torch.cat([enc, null.expand_as(enc)]).to(gpu_device)
    t = torch.tensor([0.625], dtype=torch.float32, device=gpu_device)
    rt.set_condition(encc)
    full = rt.forward(xt, ctx, t).float().clone()
    rt.set_uniform_rows(B)
    fast = rt.forward(xt, ctx, t).float()
    torch.cuda.synchronize()
    assert torch.equal(fast[:B], full[:B])                      # conditional rows untouched
    assert rel_l2(fast[B:].cpu(), full[B:].cpu()) < 2e-3          # closed form vs full (bf16 rounding)
    rt.set_uniform_rows(2 * B)                                    # off again
    again = rt.forward(xt, ctx, t).float()
    torch.cuda.synchronize()
    assert torch.equal(again, full)
    rt.close()


def test_weight_reload_matches_fresh_handle(gpu_device):
    """LoRA re-pack hook (§8f row 3): re-loading changed weights into a live handle
    (acehip.integration.refresh_decoder_weights) equals a handle built from them."""
    from acehip.dit import DiTRuntime
    cfg = DiTConfig.tiny(layers=2, window=8)
    W1 = {k: v.to(gpu_device, torch.bfloat16) for k, v in synth_dit_weights(cfg, seed=1, mode="parity").items()}
    W2 = {k: v.to(gpu_device, torch.bfloat16) for k, v in synth_dit_weights(cfg, seed=2, mode="parity").items()}
    g = torch.Generator().manual_seed(9)
    xt = torch.randn(1, 40, 64, generator=g).bfloat16().to(gpu_device)
    ctx = torch.randn(1, 40, 128, generator=g).bfloat16().to(gpu_device)
    enc = torch.randn(1, 12, cfg.hidden_size, generator=g).bfloat16().to(gpu_device)
    t = torch.tensor([0.5], dtype=torch.float32, device=gpu_device)
    a = DiTRuntime(cfg, 0, max_S=32, max_Bc=1, max_Lenc=16)
    a.load(W1)
    a.load(W2)                       # the refresh path
    a.set_condition(enc)
    b = DiTRuntime(cfg, 0, max_S=32, max_Bc=1, max_Lenc=16)
    b.load(W2)
    b.set_condition(enc)
    va, vb = a.forward(xt, ctx, t), b.forward(xt, ctx, t)
    torch.cuda.synchronize()
    assert torch.equal(va, vb)
    a.close(); b.close()


@pytest.mark.parametrize("M,N,K", [(125, 2048, 6144), (125, 12288, 2048), (250, 4096, 2048), (61, 256, 1024),
                                   (1, 2048, 2048), (16, 4096, 2048), (128, 2048, 2048), (129, 2048, 6144),
                                   (256, 12288, 2048), (200, 2048, 1088), (300, 2048, 2048)])
def test_gemm_splitk_small_m(gpu_device, M, N, K):
    """Small-M paths (short songs / turbo): the production dispatch (variant -1: the
    128×128 / 128×64 split-K path, or whole-K 128×64 tiles for the M ≤ 128 SwiGLU) with
    store, residual and SwiGLU epilogues."""
    ff = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(gpu_device, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * 0.02).to(gpu_device, torch.bfloat16)
    b = torch.randn(N, generator=g).to(gpu_device, torch.bfloat16)
    ref = A.float() @ W.float().t()
    C = torch.empty(M, N, device=gpu_device, dtype=torch.bfloat16)
    ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(C), N, M, N, K, ff.ptr(b), EPI_STORE,
                                          -1, ff.stream_ptr()))
    torch.cuda.synchronize()
    assert rel_l2(C.float().cpu(), (ref + b.float()).cpu()) < 5e-3
    R = torch.randn(M, N, generator=g).to(gpu_device, torch.bfloat16)
    C2 = R.clone()
    ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(C2), N, M, N, K, None, EPI_RES, -1,
                                          ff.stream_ptr()))
    torch.cuda.synchronize()
    assert rel_l2(C2.float().cpu(), (R.float() + ref.bfloat16().float()).cpu()) < 5e-3
    Cs = torch.empty(M, N // 2, device=gpu_device, dtype=torch.bfloat16)
    ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(Cs), N // 2, M, N, K, None,
                                          EPI_SWIGLU, -1, ff.stream_ptr()))
    torch.cuda.synchronize()
    y = ref.bfloat16().float().view(M, N // 64, 2, 32)
    gate, up = y[:, :, 0, :].reshape(M, N // 2), y[:, :, 1, :].reshape(M, N // 2)
    assert rel_l2(Cs.float().cpu(), (torch.nn.functional.silu(gate).bfloat16().float() * up).cpu()) < 1e-2


def test_forward_graph_replay_matches_eager(gpu_device):
    """acehip_dit_set_graph: the captured layer-stack graph gives bit-identical outputs to
    eager launches across new t / xt / out pointers, a new condition of the same shape,
    a sequence-length change (re-capture) and the CFG uniform-row toggle."""
    from acehip.dit import DiTRuntime
    cfg = DiTConfig.tiny(layers=4, window=8)
    W = {k: v.to(gpu_device, torch.bfloat16) for k, v in synth_dit_weights(cfg, seed=4, mode="parity").items()}
    g = torch.Generator().manual_seed(11)
    rt = DiTRuntime(cfg, 0, max_S=64, max_Bc=4, max_Lenc=40)
    rt.load(W)

    def both(xt, ctx, t):
        rt.use_graph(False)
        a = rt.forward(xt, ctx, t).clone()
        rt.use_graph(True)
        b = rt.forward(xt, ctx, t)
        c = rt.forward(xt, ctx, t)          # replay of the same capture
        torch.cuda.synchronize()
        assert torch.equal(a, b) and torch.equal(a, c)
        return a

    for T, Le, seed_t in [(100, 37, 0.625), (100, 37, 0.25), (77, 37, 0.5), (100, 21, 0.9)]:
        xt = torch.randn(2, T, 64, generator=g).bfloat16().to(gpu_device)
        ctx = torch.randn(2, T, 128, generator=g).bfloat16().to(gpu_device)
        enc = torch.randn(2, Le, cfg.hidden_size, generator=g).bfloat16()
        null = torch.randn(1, 1, cfg.hidden_size, generator=g).bfloat16()
        rt.set_condition(torch.cat([enc, null.expand_as(enc)]).to(gpu_device))
        t = torch.tensor([seed_t], dtype=torch.float32, device=gpu_device)
        both(xt, ctx, t)
        rt.set_uniform_rows(2)
        both(xt, ctx, t)
    rt.close()


def test_graph_replay_single_streamk_layer(gpu_device, monkeypatch):
    """A captured forward whose body holds exactly ONE stream-K launch (advisor r05: with per-launch
    epochs baked into the graph, each replay would have read the previous replay's flags as
    already published).  Two layers (band, then full at S = 1600: 13 q-blocks × 2 rows = 26 units of
    25 KV tiles on a 7-CU plan → stream-K), replayed several times: bit-identical to eager."""
    from acehip.dit import DiTRuntime
    set_knob(monkeypatch, "ACEHIP_ATTN_CUS", "7")
    set_knob(monkeypatch, "ACEHIP_ATTN_STREAMK", "1")
    cfg = DiTConfig.tiny(layers=2, window=8)
    W = {k: v.to(gpu_device, torch.bfloat16) for k, v in synth_dit_weights(cfg, seed=5, mode="parity").items()}
    g = torch.Generator().manual_seed(12)
    rt = DiTRuntime(cfg, 0, max_S=1600, max_Bc=2, max_Lenc=24)
    rt.load(W)
    T = 3200
    enc = torch.randn(2, 24, cfg.hidden_size, generator=g).bfloat16().to(gpu_device)
    rt.set_condition(enc)
    t = torch.tensor([0.5], dtype=torch.float32, device=gpu_device)
    outs = []
    for graph in (False, True, True, True):
        xt = torch.randn(1, T, 64, generator=torch.Generator().manual_seed(3)).bfloat16().to(gpu_device)
        ctx = torch.randn(1, T, 128, generator=torch.Generator().manual_seed(4)).bfloat16().to(gpu_device)
        rt.use_graph(graph)
        outs.append(rt.forward(xt, ctx, t).clone())
        torch.cuda.synchronize()
    rt.close()
    assert torch.isfinite(outs[0].float()).all()
    for o in outs[1:]:
        assert torch.equal(outs[0], o)


@pytest.mark.parametrize("M,N,K,epi", [(125, 12288, 2048, EPI_SWIGLU), (128, 12288, 2048, EPI_SWIGLU),
                                       (77, 1024, 512, EPI_SWIGLU), (1, 12288, 2048, EPI_SWIGLU),
                                       (125, 2048, 6144, EPI_RES), (125, 4096, 2048, EPI_STORE),
                                       (250, 4096, 2048, EPI_STORE), (125, 2048, 2048, EPI_RES)])
def test_gemm_small_m_paths(gpu_device, monkeypatch, M, N, K, epi):
    """Turbo / short-song GEMMs (M ≤ 256): SwiGLU of one 128-row chunk on whole-K 128×64 tiles
    with the epilogue fused (ACEHIP_SMALLM_WHOLEK: 2 default, + DMA helper waves; 1 without),
    and the split-K path on 64- or 128-column tiles (ACEHIP_SPLITK_BN, default 64): every
    variant vs fp32 torch."""
    ff = _lib()
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, generator=g).to(gpu_device, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * 0.02).to(gpu_device, torch.bfloat16)
    ncol = N // 2 if epi == EPI_SWIGLU else N
    C0 = torch.randn(M, ncol, generator=g).to(gpu_device, torch.bfloat16)
    ref = A.float() @ W.float().t()
    if epi == EPI_SWIGLU:
        y = ref.bfloat16().float().view(M, N // 64, 2, 32)
        gate, up = y[:, :, 0, :].reshape(M, ncol), y[:, :, 1, :].reshape(M, ncol)
        want, tol = torch.nn.functional.silu(gate).bfloat16().float() * up, 1e-2
        knobs = [{}, {"ACEHIP_SMALLM_WHOLEK": "1"}, {"ACEHIP_SMALLM_WHOLEK": "0"},
                 {"ACEHIP_SMALLM_WHOLEK": "0", "ACEHIP_SPLITK_BN": "128"}]
    else:
        want, tol = ref + (C0.float() if epi == EPI_RES else 0), (1e-2 if epi == EPI_RES else 5e-3)
        knobs = [{}, {"ACEHIP_SPLITK_BN": "64"}, {"ACEHIP_SPLITK_BN": "128"}]
    for kn in knobs:
        for k, v in kn.items():
            set_knob(monkeypatch, k, v)
        C = C0.clone()
        ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(C), ncol, M, N, K, None, epi, -1,
                                              ff.stream_ptr()))
        torch.cuda.synchronize()
        assert torch.isfinite(C.float()).all(), kn
        err = rel_l2(C.float().cpu(), want.cpu()) if epi != EPI_RES else \
            rel_l2((C.float() - C0.float()).cpu(), ref.cpu())
        assert err < tol, (kn, err)
        for k in kn:
            monkeypatch.delenv(k)
        ff.reload_knobs()


@pytest.mark.parametrize("M,N,K,epi", [(6000, 12288, 2048, EPI_SWIGLU), (15000, 12288, 2048, EPI_SWIGLU),
                                       (6000, 12288, 2048, EPI_STORE)])
def test_gemm_tail_split(gpu_device, monkeypatch, M, N, K, epi):
    """Ping-pong grids with a small last round run their tail rows as one round of 128x128
    tiles (gemm_tail_split): vs fp32 torch, and vs the unsplit launch."""
    ff = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + K)
    A = torch.randn(M, K, generator=g).to(gpu_device, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * 0.02).to(gpu_device, torch.bfloat16)
    ref = A.float() @ W.float().t()
    ncol = N // 2 if epi == EPI_SWIGLU else N

    def run(split):
        set_knob(monkeypatch, "ACEHIP_GEMM_TAILSPLIT", "1" if split else "0")
        C = torch.full((M, ncol), float("nan"), device=gpu_device, dtype=torch.bfloat16)
        ff.check(ff.lib().acehip_gemm_bf16_ex(ff.ptr(A), K, ff.ptr(W), K, ff.ptr(C), ncol, M, N, K, None, epi, -1,
                                              ff.stream_ptr()))
        torch.cuda.synchronize()
        return C.float()

    on, off = run(True), run(False)
    assert torch.isfinite(on).all()
    if epi == EPI_SWIGLU:
        y = ref.bfloat16().float().view(M, N // 64, 2, 32)
        gate, up = y[:, :, 0, :].reshape(M, ncol), y[:, :, 1, :].reshape(M, ncol)
        want = torch.nn.functional.silu(gate).bfloat16().float() * up
        tol = 1e-2
    else:
        want, tol = ref, 5e-3
    assert rel_l2(on.cpu(), want.cpu()) < tol
    assert rel_l2(on.cpu(), off.cpu()) < tol


def test_cfg_row_dedup_matches_full(gpu_device, monkeypatch):
    """CFG rows reading the same xt/ctx row at one broadcast t are identical until the first
    cross-attention: proj_in + layer 0's self-attention run on row 0 and are copied
    (ACEHIP_DIT_DEDUP).  Same result as computing both rows (kernel rounding aside)."""
    from acehip.dit import DiTRuntime
    cfg = DiTConfig.tiny(layers=4, window=16)
    W = {k: v.to(gpu_device, torch.bfloat16) for k, v in synth_dit_weights(cfg, seed=6, mode="parity").items()}
    g = torch.Generator().manual_seed(21)
    rt = DiTRuntime(cfg, 0, max_S=256, max_Bc=2, max_Lenc=64)
    rt.load(W)
    xt = torch.randn(1, 401, 64, generator=g).bfloat16().to(gpu_device)
    ctx = torch.randn(1, 401, 128, generator=g).bfloat16().to(gpu_device)
    enc = torch.randn(2, 50, cfg.hidden_size, generator=g).bfloat16().to(gpu_device)
    rt.set_condition(enc)
    t = torch.tensor([0.7], dtype=torch.float32, device=gpu_device)
    set_knob(monkeypatch, "ACEHIP_DIT_DEDUP", "0")
    full = rt.forward(xt, ctx, t).float().clone()
    set_knob(monkeypatch, "ACEHIP_DIT_DEDUP", "1")
    dd = rt.forward(xt, ctx, t).float()
    torch.cuda.synchronize()
    assert rel_l2(dd.cpu(), full.cpu()) < 2e-3
    # a per-row t (t_stride 1) must not take the shortcut: rows then differ
    t2 = torch.tensor([0.7, 0.3], dtype=torch.float32, device=gpu_device)
    a = rt.forward(xt, ctx, t2).float()
    set_knob(monkeypatch, "ACEHIP_DIT_DEDUP", "0")
    b = rt.forward(xt, ctx, t2).float()
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    rt.close()


def test_production_cfg_path_all_shortcuts(gpu_device, monkeypatch):
    """The production CFG call for one song — Bx = 1, Bc = 2, null condition rows
    (null_condition_emb.expand, base:1907) with set_uniform_rows(1) — runs the layer-0 row
    dedup, the closed-form null-row cross-attention and the null-row add fused into the MLP
    norm together: vs all three off (ACEHIP_DIT_DEDUP=0, ACEHIP_FUSE_ROWADD=0, full
    cross-attention), and vs the bf16 CPU oracle on the expanded condition."""
    from acehip.dit import DiTRuntime
    cfg = DiTConfig.tiny(layers=4, window=16)
    W = synth_dit_weights(cfg, seed=8, mode="parity")
    g = torch.Generator().manual_seed(31)
    T, Lenc = 301, 45
    xt = torch.randn(1, T, 64, generator=g).bfloat16()
    ctx = torch.randn(1, T, 128, generator=g).bfloat16()
    enc = torch.randn(1, Lenc, cfg.hidden_size, generator=g).bfloat16()
    null = torch.randn(1, 1, cfg.hidden_size, generator=g).bfloat16()
    encc = torch.cat([enc, null.expand_as(enc)])
    t = torch.tensor([0.55], dtype=torch.bfloat16)
    rt = DiTRuntime(cfg, 0, max_S=256, max_Bc=2, max_Lenc=64)
    rt.load({k: v.to(gpu_device, torch.bfloat16) for k, v in W.items()})
    rt.set_condition(encc.to(gpu_device))
    x_d, c_d, t_d = xt.to(gpu_device), ctx.to(gpu_device), t.float().to(gpu_device)
    rt.set_uniform_rows(1)
    fast = rt.forward(x_d, c_d, t_d).float().clone()
    set_knob(monkeypatch, "ACEHIP_DIT_DEDUP", "0")
    set_knob(monkeypatch, "ACEHIP_FUSE_ROWADD", "0")
    rt.set_uniform_rows(2)                                  # off: full cross-attention for every row
    full = rt.forward(x_d, c_d, t_d).float()
    torch.cuda.synchronize()
    assert rel_l2(fast.cpu(), full.cpu()) < 3e-3
    Wb = {k: v.bfloat16() for k, v in W.items()}
    with torch.no_grad():
        ref = dit_oracle.dit_forward(Wb, cfg, torch.cat([xt, xt]), t.expand(2), t.expand(2), encc,
                                     torch.cat([ctx, ctx])).float()
    assert rel_l2(fast.cpu(), ref) <= TOL_REL and cosine(fast.cpu(), ref) >= TOL_COS
    rt.close()


def test_null_row_add_fused_into_norm(gpu_device, monkeypatch):
    """The CFG null rows' constant cross-O output added inside the MLP RMSNorm pass
    (RowAdd) is bit-identical to the separate add_row_bcast launch."""
    from acehip.dit import DiTRuntime
    cfg = DiTConfig.tiny(layers=4, window=8)
    W = {k: v.to(gpu_device, torch.bfloat16) for k, v in synth_dit_weights(cfg, seed=8, mode="parity").items()}
    g = torch.Generator().manual_seed(13)
    rt = DiTRuntime(cfg, 0, max_S=128, max_Bc=4, max_Lenc=40)
    rt.load(W)
    B, T, Le = 2, 203, 33
    xt = torch.randn(B, T, 64, generator=g).bfloat16().to(gpu_device)
    ctx = torch.randn(B, T, 128, generator=g).bfloat16().to(gpu_device)
    enc = torch.randn(B, Le, cfg.hidden_size, generator=g).bfloat16()
    null = torch.randn(1, 1, cfg.hidden_size, generator=g).bfloat16()
    rt.set_condition(torch.cat([enc, null.expand_as(enc)]).to(gpu_device))
    rt.set_uniform_rows(B)
    t = torch.tensor([0.4], dtype=torch.float32, device=gpu_device)
    set_knob(monkeypatch, "ACEHIP_FUSE_ROWADD", "0")
    sep = rt.forward(xt, ctx, t).clone()
    set_knob(monkeypatch, "ACEHIP_FUSE_ROWADD", "1")
    fused = rt.forward(xt, ctx, t)
    torch.cuda.synchronize()
    assert torch.equal(sep, fused)
    rt.close()


@pytest.mark.parametrize("graph", [False, True])
def test_forward_step_matches_forward(gpu_device, graph):
    """acehip_dit_set_timesteps + forward_step(i) (timestep MLPs of the whole schedule in one
    pass, 40 steps = 3 row chunks) is bit-identical to forward(t[i]) for every step, with and
    without the HIP graph; t_r != t exercises the second (t − t_r) embedding."""
    from acehip.dit import DiTRuntime
    cfg = DiTConfig.tiny(layers=2, window=16)
    W = {k: v.to(gpu_device, torch.bfloat16) for k, v in synth_dit_weights(cfg, seed=9, mode="parity").items()}
    g = torch.Generator().manual_seed(41)
    rt = DiTRuntime(cfg, 0, max_S=128, max_Bc=2, max_Lenc=64)
    rt.load(W)
    rt.use_graph(graph)
    xt = torch.randn(1, 201, 64, generator=g).bfloat16().to(gpu_device)
    ctx = torch.randn(1, 201, 128, generator=g).bfloat16().to(gpu_device)
    rt.set_condition(torch.randn(2, 30, cfg.hidden_size, generator=g).bfloat16().to(gpu_device))
    n = 40
    t = torch.linspace(1.0, 0.05, n, device=gpu_device, dtype=torch.float32)
    t_r = (t * 0.5).contiguous()
    rt.set_timesteps(t, t_r)
    for i in [0, 1, 15, 16, 17, 39]:
        a = rt.forward(xt, ctx, t[i:i + 1], t_r[i:i + 1]).clone()
        b = rt.forward_step(xt, ctx, i)
        torch.cuda.synchronize()
        assert torch.equal(a, b), i
    with pytest.raises(RuntimeError):
        rt.forward_step(xt, ctx, n)                  # outside the schedule
    rt.close()


def _small_m_cfg():
    # the real width (K = 2048 / 4096: ≥ 8 K-tiles, so the short-song GEMMs take the split-K
    # path, and D = 2048 puts the deferred-epilogue norm on its 4-waves-per-row kernel)
    return DiTConfig(hidden_size=2048, intermediate_size=4096, num_hidden_layers=3, num_attention_heads=16,
                     num_key_value_heads=8, head_dim=128, sliding_window=16)


@pytest.mark.parametrize("mode", ["turbo", "cfg", "null_only"])
def test_splitk_epilogue_fused_into_consumers(gpu_device, monkeypatch, mode):
    """Short songs (M = Bc·S ≤ 256): every projection runs on the split-K path; its epilogue is
    folded into the consumer — head_post reads the QKV / cross-Q partials, and the residual
    epilogues of O, cross-O and down are applied by the next RMSNorm pass (gemm(..., defer)).
    Bit-identical to the separate splitk_epilogue_kernel launches (ACEHIP_SPLITK_FUSE=0), for
    turbo (Bc = 1), the CFG pair with closed-form null rows + layer-0 dedup, and a condition
    whose every row is the null row (no cross-attention at all); turbo also vs the oracle."""
    from acehip.dit import DiTRuntime
    cfg = _small_m_cfg()
    W = synth_dit_weights(cfg, seed=17, mode="parity")
    g = torch.Generator().manual_seed(5)
    T, Lenc = 181, 37
    xt = torch.randn(1, T, 64, generator=g).bfloat16()
    ctx = torch.randn(1, T, 128, generator=g).bfloat16()
    enc = torch.randn(1, Lenc, cfg.hidden_size, generator=g).bfloat16()
    null = torch.randn(1, 1, cfg.hidden_size, generator=g).bfloat16().expand_as(enc)
    rt = DiTRuntime(cfg, 0, max_S=128, max_Bc=2, max_Lenc=64)
    rt.load({k: v.to(gpu_device, torch.bfloat16) for k, v in W.items()})
    if mode == "turbo":
        rt.set_condition(enc.to(gpu_device))
    elif mode == "cfg":
        rt.set_condition(torch.cat([enc, null]).to(gpu_device))
        rt.set_uniform_rows(1)
    else:
        rt.set_condition(null.contiguous().to(gpu_device))
        rt.set_uniform_rows(0)
    t = torch.tensor([0.6], dtype=torch.float32, device=gpu_device)
    x_d, c_d = xt.to(gpu_device), ctx.to(gpu_device)
    set_knob(monkeypatch, "ACEHIP_SPLITK_FUSE", "0")
    sep = rt.forward(x_d, c_d, t).clone()
    set_knob(monkeypatch, "ACEHIP_SPLITK_FUSE", "1")
    fused = rt.forward(x_d, c_d, t)
    torch.cuda.synchronize()
    assert torch.equal(sep, fused)
    if mode == "turbo":
        Wb = {k: v.bfloat16() for k, v in W.items()}
        tb = torch.tensor([0.6], dtype=torch.bfloat16)
        with torch.no_grad():
            ref = dit_oracle.dit_forward(Wb, cfg, xt, tb, tb, enc, ctx).float()
        out = fused.float().cpu()
        assert rel_l2(out, ref) <= TOL_REL and cosine(out, ref) >= TOL_COS
    rt.close()


def test_cross_kv_grouped_gemms(gpu_device, monkeypatch):
    """set_condition's cross K/V projections run as GEMMs over groups of kv_group layers (the
    group bounded by a scratch budget: at the production handle's max_Bc 16 x max_Lenc 2048 it
    is 2 layers per GEMM).  ACEHIP_KV_GROUP_KIB shrinks the budget so a tiny 5-layer handle runs
    groups of 2, 2, 1 (ldkv = G·2·kvd with a partial last group) — the forward must equal the
    one-group handle's and the oracle's."""
    from acehip.dit import DiTRuntime
    cfg = DiTConfig.tiny(layers=5, window=8)
    W = synth_dit_weights(cfg, seed=17, mode="parity")
    g = torch.Generator().manual_seed(17)
    B, T, Le = 2, 60, 32
    xt = torch.randn(B, T, 64, generator=g).bfloat16().to(gpu_device)
    ctx = torch.randn(B, T, 128, generator=g).bfloat16().to(gpu_device)
    enc = torch.randn(B, Le, cfg.hidden_size, generator=g).bfloat16().to(gpu_device)
    t = torch.tensor([0.4375, 0.8125], dtype=torch.float32, device=gpu_device)
    outs = []
    for kib in (None, 64):                       # per layer: 2·32·2·128·2 B = 32 KiB → groups of 2
        if kib:
            set_knob(monkeypatch, "ACEHIP_KV_GROUP_KIB", kib)
        rt = _runtime(cfg, W, gpu_device, max_S=32, max_Bc=2, max_Lenc=Le)
        rt.set_condition(enc)
        outs.append(rt.forward(xt, ctx, t).float().cpu())
        torch.cuda.synchronize()
        rt.close()
    Wb = {k: v.bfloat16() for k, v in W.items()}
    with torch.no_grad():
        ref = dit_oracle.dit_forward(Wb, cfg, xt.cpu(), t.cpu().bfloat16(), t.cpu().bfloat16(), enc.cpu(),
                                     ctx.cpu()).float()
    assert rel_l2(outs[1], outs[0]) < 1e-3, rel_l2(outs[1], outs[0])
    assert rel_l2(outs[1], ref) <= TOL_REL and cosine(outs[1], ref) >= TOL_COS


@pytest.mark.parametrize("cus,B,H,KV,Sq,Sk", [(16, 2, 4, 2, 700, 1600), (20, 2, 4, 2, 700, 3100), (0, 2, 16, 8, 3000, 3000),
                                              (0, 2, 16, 8, 7500, 7500), (7, 1, 4, 2, 1000, 1700), (3, 1, 2, 1, 450, 1600),
                                              (512, 2, 16, 8, 7500, 7500), (384, 2, 16, 8, 3000, 3000)])
def test_attention_streamk(gpu_device, monkeypatch, cus, B, H, KV, Sq, Sk):
    """Stream-K rounds (ACEHIP_ATTN_STREAMK=1) for unmasked full / cross layers: the units' KV tiles
    as one sequence split evenly over the workgroups; a split unit's pieces meet through a
    last-arriver ticket and the folder folds them in workgroup order.  ACEHIP_ATTN_CUS shrinks the
    grid so units span 2-3 workgroups; cus = 0 is the real 240 s full / cross shape; cus = 384 / 512
    plan more workgroups than the device holds at once (advisor r05: the old flag spin needed the
    whole grid resident) — no workgroup waits for another, so those must be exact too.  vs fp32,
    and bit-identical across launches whichever piece folds."""
    if cus:
        set_knob(monkeypatch, "ACEHIP_ATTN_CUS", str(cus))
    set_knob(monkeypatch, "ACEHIP_ATTN_STREAMK", "1")
    set_knob(monkeypatch, "ACEHIP_ATTN_PW", "2")
    ff = _lib()
    g = torch.Generator(device="cpu").manual_seed(Sq + Sk + cus)
    q = torch.randn(B, H, Sq, 128, generator=g).to(gpu_device, torch.bfloat16)
    k = torch.randn(B, KV, Sk, 128, generator=g).to(gpu_device, torch.bfloat16)
    v = torch.randn(B, KV, Sk, 128, generator=g).to(gpu_device, torch.bfloat16)
    outs = []
    for _ in range(3):
        o = torch.full((B, Sq, H * 128), float("nan"), device=gpu_device, dtype=torch.bfloat16)
        ff.check(ff.lib().acehip_attention_bf16(ff.ptr(q), ff.ptr(k), ff.ptr(v), ff.ptr(o), B, H, KV, Sq, Sk, -1,
                                                1 / math.sqrt(128), ff.stream_ptr()))
        torch.cuda.synchronize()
        outs.append(o)
    ref = _attn_ref(q, k, v, -1).transpose(1, 2).reshape(B, Sq, H * 128)
    assert torch.isfinite(outs[0].float()).all()
    assert rel_l2(outs[0].float().cpu(), ref.float().cpu()) < 1e-2
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
