"""GPU parity of the condition encoders (§8f row 1) through the C ABI:
masked attention kernel vs fp32 torch SDPA with the reference's additive mask,
lyric / timbre encoders and the packed AceStepConditionEncoder output vs the
reference's golden vectors (tools/make_golden.py gen_condenc).

Tolerance (same contract as the DiT): bf16 HIP vs reference
rel-L2 <= 2.5 %, cosine >= 0.999; masks and packing order exact."""
import pytest
import torch

from conftest import cosine, golden_manifest, load_golden, rel_l2

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
    reference fixtures (tools/make_golden.py gen_tokenizer); codes may flip at a rounding
    boundary in bf16, so indices are compared by agreement rate."""
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
