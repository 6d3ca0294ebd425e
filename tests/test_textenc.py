"""Qwen3 text encoder (Qwen3-Embedding-0.6B, the reference's
``text_encoder``, conditioning_embed.py:71-79).  Golden vectors from transformers'
``Qwen3Model`` run in this container (tools/make_golden_text.py) on the seeded synthetic
weights regenerated here; the oracle restatement (oracle.condenc_oracle.text_encoder) is
pinned against them on CPU, the HIP path (acehip.condition.TextEncoder: causal
encoder-stack runtime) on the GPU."""
import pytest
import torch
from safetensors import safe_open

from conftest import set_knob, GOLDEN, cosine, load_golden, rel_l2

from acehip.config import DiTConfig
from acehip.weights import synth_text_encoder_weights
from oracle import condenc_oracle

TOL_REL, TOL_COS = 0.025, 0.999


def _setup():
    with safe_open(f"{GOLDEN}/textenc_tiny.safetensors", "pt") as f:
        meta = f.metadata()
    cfg = DiTConfig(hidden_size=int(meta["hidden_size"]), intermediate_size=int(meta["intermediate_size"]),
                    num_hidden_layers=int(meta["num_hidden_layers"]),
                    num_attention_heads=int(meta["num_attention_heads"]),
                    num_key_value_heads=int(meta["num_key_value_heads"]), head_dim=int(meta["head_dim"]),
                    rms_norm_eps=float(meta["rms_norm_eps"]), rope_theta=float(meta["rope_theta"]))
    W = synth_text_encoder_weights(cfg, int(meta["vocab_size"]), seed=7, mode="parity")
    return cfg, W, load_golden("textenc_tiny")


@pytest.mark.parametrize("tag", ["a", "b"])
def test_text_encoder_oracle_vs_transformers(tag):
    cfg, W, g = _setup()
    ids = g[f"ids_{tag}"]
    with torch.no_grad():
        o32 = condenc_oracle.text_encoder(W, cfg, ids)
        o16 = condenc_oracle.text_encoder({k: v.bfloat16() for k, v in W.items()}, cfg, ids)
    assert rel_l2(o32, g[f"out_f32_{tag}"]) < 1e-5
    assert rel_l2(o16.float(), g[f"out_bf16_{tag}"].float()) < 0.01


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["a", "b"])
def test_text_encoder_hip_vs_transformers(gpu_device, tag):
    from acehip.condition import TextEncoder
    cfg, W, g = _setup()
    te = TextEncoder(cfg, device=gpu_device.index or 0, max_batch=2, max_tokens=256)
    te.load({k: v.to(gpu_device) for k, v in W.items()})
    ids = g[f"ids_{tag}"].to(gpu_device)
    out = te(input_ids=ids, lyric_attention_mask=None).last_hidden_state
    emb = te.embed_tokens(ids)
    torch.cuda.synchronize()
    ref = g[f"out_bf16_{tag}"].float()
    assert rel_l2(out.float().cpu(), ref) <= TOL_REL, rel_l2(out.float().cpu(), ref)
    assert cosine(out.float().cpu(), ref) >= TOL_COS
    assert torch.equal(emb.cpu(), torch.nn.functional.embedding(ids.cpu(), W["embed_tokens.weight"].bfloat16()))
    te.close()


@pytest.mark.gpu
def test_text_encoder_real_width_splitk_fusion(gpu_device, monkeypatch):
    """The real Qwen3-0.6B width (D = 1024, F = 3072; 3 of its 28 layers) at 128 tokens: the
    O / down GEMMs take the split-K path and their residual epilogue is applied by the next
    RMSNorm (2 waves per row).  Bit-identical to the separate split-K epilogue launches
    (ACEHIP_SPLITK_FUSE=0), and within the bf16 tolerance of the oracle."""
    from acehip.condition import TextEncoder
    from acehip.config import DiTConfig
    from acehip.weights import synth_text_encoder_weights
    from oracle import condenc_oracle
    cfg = DiTConfig(**dict(TextEncoder.QWEN3_06B, num_hidden_layers=3))
    W = synth_text_encoder_weights(cfg, 300, seed=4, mode="parity")
    te = TextEncoder(cfg, device=gpu_device.index or 0, max_batch=1, max_tokens=256)
    te.load({k: v.to(gpu_device) for k, v in W.items()})
    ids = torch.randint(0, 300, (1, 128), generator=torch.Generator().manual_seed(9)).to(gpu_device)
    set_knob(monkeypatch, "ACEHIP_SPLITK_FUSE", "0")
    sep = te(input_ids=ids).last_hidden_state.clone()
    set_knob(monkeypatch, "ACEHIP_SPLITK_FUSE", "1")
    fused = te(input_ids=ids).last_hidden_state
    torch.cuda.synchronize()
    assert torch.equal(sep, fused)
    Wb = {k: v.bfloat16() for k, v in W.items()}
    with torch.no_grad():
        ref = condenc_oracle.text_encoder(Wb, cfg, ids.cpu()).float()
    out = fused.float().cpu()
    assert rel_l2(out, ref) <= TOL_REL and cosine(out, ref) >= TOL_COS
    te.close()
