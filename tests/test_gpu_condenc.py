"""GPU parity of the condition encoders (§8f row 1) through the C ABI:
masked attention kernel vs fp32 torch SDPA with the reference's additive mask,
lyric / timbre encoders and the packed AceStepConditionEncoder output vs the
reference's golden vectors (tools/make_golden.py gen_condenc).

Tolerance (same contract as the DiT): bf16 HIP vs reference
rel-L2 <= 2.5 %, cosine >= 0.999; masks and packing order exact."""
import pytest
import torch

from conftest import cosine, golden_manifest, load_golden, rel_l2, set_knob

from acehip.config import DiTConfig
from acehip.weights import synth_condenc_weights
from oracle import condenc_oracle as co

pytestmark = pytest.mark.gpu

TOL_REL, TOL_COS = 0.025, 0.999


@pytest.mark.parametrize("H,KV,S,window,valid", [(2, 1, 300, 8, [300, 37]), (16, 8, 200, 128, [5, 200]),
                                                  (2, 2, 130, -1, [1, 64]), (16, 8, 70, 16, [70, 3])])
def test_masked_attention(gpu_device, H, KV, S, window, valid):
    from acehip import _ffi as ff
    B = len(valid)
    g = torch.Generator().manual_seed(S + H)
    q = torch.randn(B, H, S, 128, generator=g).bfloat16()
    k = torch.randn(B, KV, S, 128, generator=g).bfloat16()
    v = torch.randn(B, KV, S, 128, generator=g).bfloat16()
    m = torch.zeros(B, S, dtype=torch.long)
    for b, n in enumerate(valid):
        m[b, :n] = 1
    mask = co.create_4d_mask(S, torch.float32, m, window if window >= 0 else None)
    rep = H // KV
    ref = torch.nn.functional.scaled_dot_product_attention(
        q.float(), k.float().repeat_interleave(rep, 1), v.float().repeat_interleave(rep, 1), attn_mask=mask,
        scale=128 ** -0.5).transpose(1, 2).reshape(B, S, H * 128)
    qd, kd, vd = (t.to(gpu_device).contiguous() for t in (q, k, v))
    km = m.to(gpu_device, torch.uint8).contiguous()
    o = torch.empty(B, S, H * 128, device=gpu_device, dtype=torch.bfloat16)
    ff.check(ff.lib().acehip_attention_masked_bf16(ff.ptr(qd), ff.ptr(kd), ff.ptr(vd), ff.ptr(o), B, H, KV, S, S,
                                                   window, 128 ** -0.5, ff.ptr(km), ff.stream_ptr()))
    torch.cuda.synchronize()
    o = o.float().cpu()
    assert rel_l2(o, ref) < 1e-2
    # rows with no admissible key: uniform over every key (finite finfo.min semantics)
    assert torch.isfinite(o).all()


@pytest.mark.parametrize("H,KV,S,valid", [(16, 8, 300, [0, 217]), (2, 1, 1000, [999, 3]), (4, 2, 77, [77, 1]),
                                           (16, 16, 250, [250, 0])])
def test_masked_attention_small(gpu_device, monkeypatch, H, KV, S, valid):
    """Key-padding-masked full attention on attn_small_kernel (ACEHIP_ATTN_SMALL_MASK, the
    encoders' short grids; KV parts through the workspace at S = 1000): against SDPA
    with the reference's additive mask — an all-masked row (valid 0) is uniform over its S keys —
    and against attn_fwd_kernel's masked mode (=0)."""
    from acehip import _ffi as ff
    B = len(valid)
    g = torch.Generator().manual_seed(S * 3 + H)
    q = torch.randn(B, H, S, 128, generator=g).bfloat16()
    k = torch.randn(B, KV, S, 128, generator=g).bfloat16()
    v = torch.randn(B, KV, S, 128, generator=g).bfloat16()
    m = torch.zeros(B, S, dtype=torch.long)
    for b, n in enumerate(valid):
        m[b, :n] = 1
    mask = co.create_4d_mask(S, torch.float32, m, None)
    rep = H // KV
    ref = torch.nn.functional.scaled_dot_product_attention(
        q.float(), k.float().repeat_interleave(rep, 1), v.float().repeat_interleave(rep, 1), attn_mask=mask,
        scale=128 ** -0.5).transpose(1, 2).reshape(B, S, H * 128)
    qd, kd, vd = (t.to(gpu_device).contiguous() for t in (q, k, v))
    km = m.to(gpu_device, torch.uint8).contiguous()
    outs = {}
    for mode in ("1", "0"):
        set_knob(monkeypatch, "ACEHIP_ATTN_SMALL_MASK", mode)
        o = torch.full((B, S, H * 128), float("nan"), device=gpu_device, dtype=torch.bfloat16)
        ff.check(ff.lib().acehip_attention_masked_bf16(ff.ptr(qd), ff.ptr(kd), ff.ptr(vd), ff.ptr(o), B, H, KV, S,
                                                       S, -1, 128 ** -0.5, ff.ptr(km), ff.stream_ptr()))
        torch.cuda.synchronize()
        outs[mode] = o.float().cpu()
        assert torch.isfinite(outs[mode]).all()
        assert rel_l2(outs[mode], ref) < 1e-2
    assert rel_l2(outs["1"], outs["0"]) < 1e-2


def _setup(name, gpu_device):
    from acehip.condition import ConditionEncoder
    meta = golden_manifest()["condenc"][name]
    cfg = DiTConfig(**meta["cfg"])
    g = load_golden("condenc_" + name)
    W = synth_condenc_weights(cfg, seed=meta["seed"], mode="parity")
    ce = ConditionEncoder(cfg, gpu_device.index or 0, max_batch=2, max_lyric=64, max_refs=4, max_ref_frames=32)
    ce.load({k: v.to(gpu_device, torch.bfloat16) for k, v in W.items()})
    return cfg, g, ce


@pytest.mark.parametrize("name", ["tiny_bfloat16", "tiny_float32", "full_bfloat16"])
def test_condition_encoder_vs_reference(gpu_device, name):
    cfg, g, ce = _setup(name, gpu_device)
    d = gpu_device
    lyr = ce.lyric_encoder(g["lyric"].to(d), g["lyric_mask"].to(d)).float().cpu()
    tim, tmask = ce.timbre_encoder(g["refer"].to(d), g["order"].to(d))
    enc, mask = ce(g["text"].to(d), g["text_mask"].to(d), g["lyric"].to(d), g["lyric_mask"].to(d),
                   g["refer"].to(d), g["order"].to(d))
    torch.cuda.synchronize()
    for out, ref in ((lyr, g["lyric_out"]), (tim.float().cpu(), g["timbre_out"]), (enc.float().cpu(), g["enc"])):
        assert out.shape == ref.shape
        assert rel_l2(out, ref.float()) < TOL_REL, name
        assert cosine(out, ref.float()) > TOL_COS, name
    assert torch.equal(tmask.cpu(), g["timbre_mask"])
    assert torch.equal(mask.cpu().to(torch.uint8), g["enc_mask"])
    ce.close()


def test_prepare_condition_dropin(gpu_device):
    """HipPrepareCondition (base:1607-1652) for text2music: encoder states as above,
    context = cat(src_latents, chunk_masks)."""
    from acehip.condition import HipPrepareCondition
    cfg, g, ce = _setup("tiny_bfloat16", gpu_device)
    d = gpu_device
    T = 24
    src = torch.randn(2, T, 64, device=d).bfloat16()
    cm = torch.ones(2, T, 64, device=d).bfloat16()
    pc = HipPrepareCondition(ce)
    enc, mask, ctx = pc(text_hidden_states=g["text"].to(d), text_attention_mask=g["text_mask"].to(d),
                        lyric_hidden_states=g["lyric"].to(d), lyric_attention_mask=g["lyric_mask"].to(d),
                        refer_audio_acoustic_hidden_states_packed=g["refer"].to(d),
                        refer_audio_order_mask=g["order"].to(d), hidden_states=src, attention_mask=None,
                        silence_latent=None, src_latents=src, chunk_masks=cm,
                        is_covers=torch.zeros(2, dtype=torch.long, device=d))
    torch.cuda.synchronize()
    assert rel_l2(enc.float().cpu(), g["enc"].float()) < TOL_REL
    assert torch.equal(ctx, torch.cat([src, cm], -1))
    with pytest.raises(NotImplementedError):
        pc(text_hidden_states=g["text"].to(d), text_attention_mask=g["text_mask"].to(d),
           lyric_hidden_states=g["lyric"].to(d), lyric_attention_mask=g["lyric_mask"].to(d),
           refer_audio_acoustic_hidden_states_packed=g["refer"].to(d), refer_audio_order_mask=g["order"].to(d),
           hidden_states=src, attention_mask=None, silence_latent=None, src_latents=src, chunk_masks=cm,
           is_covers=torch.ones(2, dtype=torch.long, device=d))
    ce.close()


@pytest.mark.parametrize("name", ["tiny_bfloat16", "tiny_float32"])
def test_tokenizer_detokenizer_vs_reference(gpu_device, name):
    """AttentionPooler / tokenizer (+ restated FSQ) / detokenizer on libacehip vs the
    reference fixtures (tools/make_golden.py gen_tokenizer).  The HIP pooler's bf16 z differs
    from the reference's by rounding, so a code can flip where z sits at a rounding
    boundary: indices are compared here by agreement rate; on IDENTICAL z the quantizer is
    bit-exact (test_fsq_bit_exact_exhaustive)."""
    from acehip.condition import AudioDetokenizer, AudioTokenizer
    from acehip.weights import synth_tokenizer_weights
    meta = golden_manifest()["tokenizer"][name]
    cfg = DiTConfig(**meta["cfg"])
    g = load_golden("tokenizer_" + name)
    W = {k: v.to(gpu_device, torch.bfloat16) for k, v in synth_tokenizer_weights(cfg, seed=meta["seed"],
                                                                               mode="parity").items()}
    tok = AudioTokenizer(cfg, 0, max_patches=64)
    tok.load(W)
    det = AudioDetokenizer(cfg, 0, max_patches=64)
    det.load(W)
    d = gpu_device
    pooled = tok.attention_pooler(g["pooled_in"].to(d, torch.bfloat16))
    x = g["x"].to(d, torch.bfloat16)
    quant, idx = tok(x.reshape(x.shape[0], -1, cfg.pool_window_size, x.shape[-1]))
    det_out = det(g["det_in"].to(d, torch.bfloat16))
    hints = det(g["quantized"].to(d, torch.bfloat16))
    torch.cuda.synchronize()
    for out, ref in ((pooled, g["pooled"]), (det_out, g["det_out"]), (hints, g["hints"])):
        assert out.shape == ref.shape
        assert rel_l2(out.float().cpu(), ref.float()) < TOL_REL
        assert cosine(out.float().cpu(), ref.float()) > TOL_COS
    agree = (idx.cpu() == g["indices"]).float().mean()
    assert agree > 0.9, float(agree)
    # codes -> indices -> output round trip (quantizer.get_output_from_indices, audio_codes.py:62)
    again = tok.get_output_from_indices(idx)
    torch.cuda.synchronize()
    assert torch.equal(again, quant)
    tok.close(); det.close()


def test_fsq_bit_exact_exhaustive(gpu_device):
    """FSQ on IDENTICAL inputs is index work and must be bit-exact: the HIP
    quantizer gets z in bf16 (the project_in GEMM output), so every one of the 65,280
    finite bf16 values plus ±inf is fed in every level column ([8,8,8,5,5,5],
    configuration_acestep_v15.py:152) and codes / indices must equal the restated
    vector_quantize_pytorch FSQ (oracle/condenc_oracle.py, base:1196-1200).  The rows
    are then rolled per column so each row mixes levels.  Rounding-boundary margin of
    this input set (fp64 analysis, CPU): the nearest bounded value to a .5 tie is
    4.9e-4 away — ~4000 fp32 ulps — so no tanh-ulp tie exists among bf16 inputs;
    the count of mismatches is asserted to be 0.  Then the inverse: all
    8·8·8·5·5·5 = 64,000 indices → codes equal the oracle, and codes → indices →
    codes is the identity on the device."""
    from acehip import _ffi as ff
    bits = torch.arange(0, 65536, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    vals = bits[~torch.isnan(bits.float())]
    assert vals.numel() == 65536 - 254
    nl = len(co.FSQ_LEVELS)
    zc = torch.stack([torch.roll(vals, 977 * i) for i in range(nl)], dim=1)      # [M, 6]
    M = zc.shape[0]
    z = torch.zeros(M, 128, dtype=torch.bfloat16)
    z[:, :nl] = zc
    z[:, nl:] = torch.randn(M, 128 - nl, generator=torch.Generator().manual_seed(3)).bfloat16()  # ignored
    ref_codes, ref_idx = co.fsq_quantize(zc)
    lv = (ff.c_int * nl)(*co.FSQ_LEVELS)
    zd = z.to(gpu_device).contiguous()
    codes = torch.full((M, 64), 7.0, device=gpu_device, dtype=torch.bfloat16)
    idx = torch.empty(M, device=gpu_device, dtype=torch.int32)
    ff.check(ff.lib().acehip_fsq_quantize(ff.ptr(zd), 128, M, lv, nl, ff.ptr(codes), 64, ff.ptr(idx),
                                          ff.stream_ptr()), "fsq_quantize")
    torch.cuda.synchronize()
    c, i = codes.cpu(), idx.cpu()
    mism = int((i != ref_idx).sum())
    assert mism == 0, f"{mism} index mismatches"
    assert torch.equal(c[:, :nl], ref_codes)
    assert torch.equal(c[:, nl:], torch.zeros(M, 64 - nl, dtype=torch.bfloat16))   # K padding
    # every index of the lattice -> codes (FSQ.indices_to_codes) and back
    n_idx = 1
    for L in co.FSQ_LEVELS:
        n_idx *= L
    all_idx = torch.arange(n_idx, dtype=torch.int32)
    ref_c = co.fsq_codes_from_indices(all_idx, torch.bfloat16)
    ad = all_idx.to(gpu_device)
    c2 = torch.empty(n_idx, 64, device=gpu_device, dtype=torch.bfloat16)
    ff.check(ff.lib().acehip_fsq_codes_from_indices(ff.ptr(ad), n_idx, lv, nl, ff.ptr(c2), 64, ff.stream_ptr()),
             "fsq_codes")
    torch.cuda.synchronize()
    assert torch.equal(c2[:, :nl].cpu(), ref_c)
    hw = torch.tensor([L // 2 for L in co.FSQ_LEVELS])
    basis = torch.cumprod(torch.tensor([1] + co.FSQ_LEVELS[:-1]), 0)
    back = ((c2[:, :nl].cpu().float() * hw + hw) * basis).sum(-1).round().to(torch.int32)
    assert torch.equal(back, all_idx)
    # device round trip indices -> codes -> indices: quantize the bf16 pre-image of each
    # lattice code under bound() (z = atanh((c·(L//2) + offset)/half_l) − shift)
    L = torch.tensor(co.FSQ_LEVELS, dtype=torch.float64)
    half = (L - 1) * (1 + 1e-3) / 2
    off = torch.where(L % 2 == 0, 0.5, 0.0)
    pre = torch.atanh((c2[:, :nl].cpu().double() * (L // 2) + off) / half) - torch.atanh(off / half)
    zp = torch.zeros(n_idx, 128, dtype=torch.bfloat16)
    zp[:, :nl] = pre.float().bfloat16()
    zpd = zp.to(gpu_device)
    idx2 = torch.empty(n_idx, device=gpu_device, dtype=torch.int32)
    codes2 = torch.empty(n_idx, 64, device=gpu_device, dtype=torch.bfloat16)
    ff.check(ff.lib().acehip_fsq_quantize(ff.ptr(zpd), 128, n_idx, lv, nl, ff.ptr(codes2), 64, ff.ptr(idx2),
                                          ff.stream_ptr()), "fsq_quantize")
    torch.cuda.synchronize()
    assert torch.equal(idx2.cpu(), all_idx)
    assert torch.equal(codes2.cpu(), c2.cpu())


def test_prepare_condition_cover(gpu_device):
    """prepare_condition (base:1635-1651) with a cover song: LM hints = detokenize(tokenize(src
    padded to a multiple of 5 with the silence latent))[:, :T] replace src where is_covers."""
    from acehip.condition import AudioDetokenizer, AudioTokenizer, HipPrepareCondition
    from acehip.weights import synth_tokenizer_weights
    cfg, g, ce = _setup("tiny_bfloat16", gpu_device)
    W = {k: v.to(gpu_device, torch.bfloat16) for k, v in synth_tokenizer_weights(cfg, seed=5, mode="parity").items()}
    tok, det = AudioTokenizer(cfg, 0, max_patches=32), AudioDetokenizer(cfg, 0, max_patches=32)
    tok.load(W)
    det.load(W)
    d = gpu_device
    T = 23                                      # not a multiple of the pool window: silence padding
    src = torch.randn(2, T, 64, device=d).bfloat16()
    sil = torch.randn(1, 40, 64, device=d).bfloat16()
    cm = torch.ones(2, T, 64, device=d).bfloat16()
    pc = HipPrepareCondition(ce, tokenizer=tok, detokenizer=det)
    enc, mask, ctx = pc(text_hidden_states=g["text"].to(d), text_attention_mask=g["text_mask"].to(d),
                        lyric_hidden_states=g["lyric"].to(d), lyric_attention_mask=g["lyric_mask"].to(d),
                        refer_audio_acoustic_hidden_states_packed=g["refer"].to(d),
                        refer_audio_order_mask=g["order"].to(d), hidden_states=src, attention_mask=None,
                        silence_latent=sil, src_latents=src, chunk_masks=cm,
                        is_covers=torch.tensor([1, 0], device=d))
    xp = torch.cat([src, sil[:1, :2].repeat(2, 1, 1)], dim=1)
    q, _ = tok(xp.reshape(2, -1, 5, 64))
    hints = det(q)[:, :T]
    torch.cuda.synchronize()
    assert torch.equal(ctx[0, :, :64], hints[0])
    assert torch.equal(ctx[1, :, :64], src[1])
    assert torch.equal(ctx[:, :, 64:], cm)
    ce.close(); tok.close(); det.close()


def test_overlapped_text_encoder_feeds_condition_encoder(gpu_device):
    """TextEncoder(overlap=True) runs its layers on a side stream and returns at once; the
    condition encoder queues its lyric and timbre encoders first and waits for the text
    encoder's event only before the text projector.  Same encoder states, bit for bit, as the
    synchronous text encoder (real text width, 3 Qwen3 layers)."""
    from acehip.condition import TextEncoder, await_ready
    from acehip.weights import synth_text_encoder_weights
    cfg, g, ce = _setup("full_bfloat16", gpu_device)
    d = gpu_device
    B, Lt = g["text"].shape[0], g["text"].shape[1]
    te_cfg = DiTConfig(**dict(TextEncoder.QWEN3_06B, num_hidden_layers=3))
    assert te_cfg.hidden_size == g["text"].shape[2]
    W = {k: v.to(d) for k, v in synth_text_encoder_weights(te_cfg, 300, seed=5, mode="parity").items()}
    ids = torch.randint(0, 300, (B, Lt), generator=torch.Generator().manual_seed(3)).to(d)
    outs = {}
    for ov in (False, True):
        te = TextEncoder(te_cfg, device=d.index or 0, max_batch=B, max_tokens=max(Lt, 64), overlap=ov)
        te.load(W)
        text = te(input_ids=ids).last_hidden_state
        enc, mask = ce(text, g["text_mask"].to(d), g["lyric"].to(d), g["lyric_mask"].to(d), g["refer"].to(d),
                       g["order"].to(d))
        await_ready(text)
        torch.cuda.synchronize()
        outs[ov] = (text.clone(), enc.clone(), mask.clone())
        te.close()
    for a, b in zip(outs[False], outs[True]):
        assert torch.equal(a, b)
    ce.close()


@pytest.mark.parametrize("B,H,KV,S", [(1, 16, 8, 128), (2, 16, 8, 77), (3, 4, 2, 300), (1, 2, 2, 257)])
def test_causal_attention_small(gpu_device, monkeypatch, B, H, KV, S):
    """Unmasked causal attention (the Qwen3 text encoder, 28 layers per song) on attn_small_kernel
    (ACEHIP_ATTN_SMALL_CAUSAL): each one-head x 32-row unit walks its keys up to its last row's
    diagonal.  vs fp32 SDPA with is_causal and vs attn_fwd_kernel's causal mode (knob off)."""
    import math
    from acehip import _ffi as ff
    from conftest import rel_l2, set_knob
    g = torch.Generator().manual_seed(B * 100 + S)
    q = torch.randn(B, H, S, 128, generator=g).bfloat16().to(gpu_device)
    k = torch.randn(B, KV, S, 128, generator=g).bfloat16().to(gpu_device)
    v = torch.randn(B, KV, S, 128, generator=g).bfloat16().to(gpu_device)

    def run(on):
        set_knob(monkeypatch, "ACEHIP_ATTN_SMALL_CAUSAL", "1" if on else "0")
        o = torch.full((B, S, H * 128), float("nan"), device=gpu_device, dtype=torch.bfloat16)
        ff.check(ff.lib().acehip_attention_bf16(ff.ptr(q), ff.ptr(k), ff.ptr(v), ff.ptr(o), B, H, KV, S, S, -2,
                                                1 / math.sqrt(128), ff.stream_ptr()))
        torch.cuda.synchronize()
        return o.float().cpu()

    on, off = run(True), run(False)
    rep = H // KV
    ref = torch.nn.functional.scaled_dot_product_attention(
        q.float(), k.float().repeat_interleave(rep, 1), v.float().repeat_interleave(rep, 1),
        is_causal=True).transpose(1, 2).reshape(B, S, H * 128).cpu()
    assert torch.isfinite(on).all()
    assert rel_l2(on, ref) < 1e-2
    assert rel_l2(on, off) < 1e-2
