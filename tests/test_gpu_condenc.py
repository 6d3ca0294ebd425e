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
