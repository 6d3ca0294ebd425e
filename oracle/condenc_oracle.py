"""CPU restatement of ACE-Step 1.5's condition encoders — TEST ORACLE ONLY.

Functional PyTorch-CPU code that reproduces, in the caller's dtype, what
``AceStepConditionEncoder.forward`` computes (reference
``acestep/models/base/modeling_acestep_v15_base.py:1527-1554``): the text
projector, the lyric encoder (:577-731), the timbre encoder (:997-1178) and
``pack_sequences`` (:138-169), plus the attention pooler (:734-859) and the
audio-token detokenizer (:862-994) built from the same encoder layer.  It is
the checker the HIP path (``acehip.condition``) is compared against; the
product path never imports it.

Weights: a flat dict keyed by the reference module-local names
(``text_projector.weight``, ``lyric_encoder.layers.0.self_attn.q_proj.weight``,
``timbre_encoder.norm.weight`` ...).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from .dit_oracle import _rotate_half, attention, rms_norm, rope_tables

Tensor = torch.Tensor


def create_4d_mask(S: int, dtype, attention_mask: Optional[Tensor], window: Optional[int]) -> Tensor:
    """create_4d_mask (base:56-135), bidirectional (is_causal=False): geometry
    |i−j| ≤ window (sliding) AND key padding (attention_mask[b, j] != 0);
    additive 0 / finfo(dtype).min, shape [B or 1, 1, S, S]."""
    idx = torch.arange(S)
    valid = torch.ones(S, S, dtype=torch.bool)
    if window is not None:
        valid = (idx[:, None] - idx[None, :]).abs() <= window
    valid = valid[None, None]
    if attention_mask is not None:
        valid = valid & attention_mask.view(attention_mask.shape[0], 1, 1, S).to(torch.bool)
    m = torch.full(valid.shape, torch.finfo(dtype).min, dtype=dtype)
    return m.masked_fill_(valid, 0.0)


def encoder_layer(W: Dict[str, Tensor], p: str, cfg, h: Tensor, mask: Tensor, cos: Tensor,
                  sin: Tensor) -> Tensor:
    """AceStepEncoderLayer.forward (base:401-440) with AceStepAttention's
    self path (base:289-371) and Qwen3MLP."""
    B, S, _ = h.shape
    hd, eps = cfg.head_dim, cfg.rms_norm_eps
    x = rms_norm(h, W[f"{p}.input_layernorm.weight"], eps)
    a = f"{p}.self_attn"
    q = rms_norm(F.linear(x, W[f"{a}.q_proj.weight"]).view(B, S, -1, hd), W[f"{a}.q_norm.weight"],
                 eps).transpose(1, 2)
    k = rms_norm(F.linear(x, W[f"{a}.k_proj.weight"]).view(B, S, -1, hd), W[f"{a}.k_norm.weight"],
                 eps).transpose(1, 2)
    v = F.linear(x, W[f"{a}.v_proj.weight"]).view(B, S, -1, hd).transpose(1, 2)
    q = q * cos + _rotate_half(q) * sin
    k = k * cos + _rotate_half(k) * sin
    o = attention(q, k, v, mask, hd ** -0.5).transpose(1, 2).reshape(B, S, -1)
    h = h + F.linear(o, W[f"{a}.o_proj.weight"])
    x = rms_norm(h, W[f"{p}.post_attention_layernorm.weight"], eps)
    m = f"{p}.mlp"
    ff = F.linear(F.silu(F.linear(x, W[f"{m}.gate_proj.weight"])) * F.linear(x, W[f"{m}.up_proj.weight"]),
                  W[f"{m}.down_proj.weight"])
    return h + ff


def encoder_body(W: Dict[str, Tensor], p: str, cfg, n_layers: int, h: Tensor,
                 attention_mask: Optional[Tensor]) -> Tensor:
    """The shared body of the lyric (base:631-722), timbre (base:1093-1173),
    pooler (base:771-854) and detokenizer (base:906-989) forwards: masks per
    layer type, RoPE positions 0..S−1, the layers, the final norm."""
    S = h.shape[1]
    dt = h.dtype
    full = create_4d_mask(S, dt, attention_mask, None)
    band = create_4d_mask(S, dt, attention_mask, cfg.sliding_window)
    cos, sin = rope_tables(S, cfg.head_dim, cfg.rope_theta, dt)
    cos, sin = cos.unsqueeze(1), sin.unsqueeze(1)
    for i in range(n_layers):
        h = encoder_layer(W, f"{p}.layers.{i}", cfg, h, band if cfg.is_sliding(i) else full, cos, sin)
    return rms_norm(h, W[f"{p}.norm.weight"], cfg.rms_norm_eps)


def lyric_encoder(W, cfg, lyric_hidden_states: Tensor, lyric_attention_mask: Tensor) -> Tensor:
    """AceStepLyricEncoder.forward (base:603-731)."""
    h = F.linear(lyric_hidden_states, W["lyric_encoder.embed_tokens.weight"],
                 W.get("lyric_encoder.embed_tokens.bias"))
    return encoder_body(W, "lyric_encoder", cfg, cfg.num_lyric_encoder_hidden_layers, h, lyric_attention_mask)


def unpack_timbre_embeddings(emb: Tensor, order: Tensor) -> Tuple[Tensor, Tensor]:
    """AceStepTimbreEncoder.unpack_timbre_embeddings (base:1023-1073): packed
    [N, d] rows → [B, max_count, d] by batch id, in packed order, + a mask."""
    N, d = emb.shape
    B = int(order.max().item() + 1)
    counts = torch.bincount(order, minlength=B)
    max_count = int(counts.max().item())
    sorted_idx = torch.argsort(order * N + torch.arange(N), stable=True)
    starts = torch.cat([torch.tensor([0]), torch.cumsum(counts, 0)[:-1]])
    pos_sorted = torch.arange(N) - starts[order[sorted_idx]]
    inv = torch.empty_like(sorted_idx)
    inv[sorted_idx] = torch.arange(N)
    pos = pos_sorted[inv]
    one_hot = F.one_hot(order * max_count + pos, num_classes=B * max_count).to(emb.dtype)
    out = (one_hot.t() @ emb).reshape(B, max_count, d)
    mask = (one_hot.sum(dim=0) > 0).long().reshape(B, max_count)
    return out, mask


def timbre_encoder(W, cfg, packed: Tensor, order: Tensor) -> Tuple[Tensor, Tensor]:
    """AceStepTimbreEncoder.forward (base:1076-1178): no padding mask; the
    special token is NOT prepended (commented out at base:1087); row 0 is the
    timbre embedding."""
    h = F.linear(packed, W["timbre_encoder.embed_tokens.weight"], W.get("timbre_encoder.embed_tokens.bias"))
    h = encoder_body(W, "timbre_encoder", cfg, cfg.num_timbre_encoder_hidden_layers, h, None)
    return unpack_timbre_embeddings(h[:, 0, :], order)


def pack_sequences(h1: Tensor, h2: Tensor, m1: Tensor, m2: Tensor) -> Tuple[Tensor, Tensor]:
    """pack_sequences (base:138-169): valid tokens first (stable), new prefix mask."""
    h = torch.cat([h1, h2], dim=1)
    m = torch.cat([m1, m2], dim=1)
    B, L, D = h.shape
    idx = m.argsort(dim=1, descending=True, stable=True)
    out = torch.gather(h, 1, idx.unsqueeze(-1).expand(B, L, D))
    lengths = m.sum(dim=1)
    return out, torch.arange(L)[None, :] < lengths[:, None]


def condition_encoder(W, cfg, text_hidden_states, text_attention_mask, lyric_hidden_states,
                      lyric_attention_mask, refer_packed, refer_order) -> Tuple[Tensor, Tensor]:
    """AceStepConditionEncoder.forward (base:1527-1554)."""
    text = F.linear(text_hidden_states, W["text_projector.weight"])
    lyric = lyric_encoder(W, cfg, lyric_hidden_states, lyric_attention_mask)
    timbre, timbre_mask = timbre_encoder(W, cfg, refer_packed, refer_order)
    enc, mask = pack_sequences(lyric, timbre, lyric_attention_mask, timbre_mask)
    return pack_sequences(enc, text, mask, text_attention_mask)


def attention_pooler(W, cfg, x: Tensor, p: str = "tokenizer.attention_pooler") -> Tensor:
    """AttentionPooler.forward (base:760-859): x [B, T, P, D] → [B, T, D]."""
    B, T, P, D = x.shape
    h = F.linear(x, W[f"{p}.embed_tokens.weight"], W.get(f"{p}.embed_tokens.bias"))
    sp = W[f"{p}.special_token"].to(h.dtype).expand(B, T, 1, -1)
    h = torch.cat([sp, h], dim=2).reshape(B * T, P + 1, D)
    h = encoder_body(W, p, cfg, cfg.num_attention_pooler_hidden_layers, h, None)
    return h[:, 0, :].reshape(B, T, D)


def detokenizer(W, cfg, x: Tensor, p: str = "detokenizer") -> Tensor:
    """AudioTokenDetokenizer.forward (base:889-994): x [B, T, D] → [B, T·P, 64]."""
    B, T, D = x.shape
    P = cfg.pool_window_size
    h = F.linear(x, W[f"{p}.embed_tokens.weight"], W.get(f"{p}.embed_tokens.bias"))
    h = h.unsqueeze(2).repeat(1, 1, P, 1) + W[f"{p}.special_tokens"].to(h.dtype).expand(B, T, -1, -1)
    h = h.reshape(B * T, P, D)
    h = encoder_body(W, p, cfg, cfg.num_attention_pooler_hidden_layers, h, None)
    h = F.linear(h, W[f"{p}.proj_out.weight"], W[f"{p}.proj_out.bias"])
    return h.reshape(B, T * P, -1)


# ---------------------------------------------------------------------------
# FSQ — vector_quantize_pytorch (>= 1.27.15, reference requirements.txt:34) is NOT
# in this container, so this is a restatement of its published algorithm
# (ResidualFSQ with num_quantizers = 1 over FSQ(levels)), PARITY UNPINNED:
#   ResidualFSQ.forward: z = project_in(x) (Linear dim→len(levels), bias);
#     quantized = FSQ(z / scale_0) · scale_0 with scale_0 = (levels−1)^0 = 1;
#     out = project_out(quantized) (Linear len(levels)→dim, bias)
#   FSQ.forward (force_quantization_f32): z.float();
#     half_l = (L−1)(1+1e-3)/2; offset = 0.5 if L even else 0; shift = atanh(offset/half_l)
#     bounded = tanh(z + shift)·half_l − offset; codes = round(bounded) / (L // 2)
#     indices = Σ_i (codes_i·(L_i//2) + L_i//2) · basis_i, basis = cumprod([1] + L[:-1])
#   codes cast back to the input dtype before project_out.
FSQ_LEVELS = [8, 8, 8, 5, 5, 5]     # configuration_acestep_v15.py:152


def fsq_quantize(z: Tensor, levels=FSQ_LEVELS) -> Tuple[Tensor, Tensor]:
    """z [..., len(levels)] (model dtype) → (codes in z's dtype, int32 indices [...])."""
    dt = z.dtype
    L = torch.tensor(levels, dtype=torch.int32)
    zf = z.float()
    half_l = (L - 1) * (1 + 1e-3) / 2
    offset = torch.where(L % 2 == 0, 0.5, 0.0)
    shift = (offset / half_l).atanh()
    bounded = (zf + shift).tanh() * half_l - offset
    hw = L // 2
    codes = bounded.round() / hw
    basis = torch.cumprod(torch.tensor([1] + levels[:-1]), dim=0, dtype=torch.int32)
    idx = ((codes * hw + hw) * basis).sum(dim=-1).round().to(torch.int32)
    return codes.to(dt), idx


def fsq_codes_from_indices(idx: Tensor, dtype, levels=FSQ_LEVELS) -> Tensor:
    """FSQ.indices_to_codes: level_i = (idx // basis_i) % L_i, code = (level − L//2)/(L//2)."""
    L = torch.tensor(levels, dtype=torch.int64)
    basis = torch.cumprod(torch.tensor([1] + levels[:-1]), dim=0)
    lv = (idx.long().unsqueeze(-1) // basis) % L
    hw = L // 2
    return ((lv - hw).float() / hw).to(dtype)


def residual_fsq(W, x: Tensor, p: str = "tokenizer.quantizer") -> Tuple[Tensor, Tensor]:
    z = F.linear(x, W[f"{p}.project_in.weight"], W[f"{p}.project_in.bias"])
    codes, idx = fsq_quantize(z)
    return F.linear(codes, W[f"{p}.project_out.weight"], W[f"{p}.project_out.bias"]), idx


def audio_tokenizer(W, cfg, x: Tensor) -> Tuple[Tensor, Tensor]:
    """AceStepAudioTokenizer.forward (base:1206-1218): x [N, T/P, P, 64] →
    (quantized [N, T/P, D], indices [N, T/P])."""
    h = F.linear(x, W["tokenizer.audio_acoustic_proj.weight"], W["tokenizer.audio_acoustic_proj.bias"])
    h = attention_pooler(W, cfg, h)
    return residual_fsq(W, h)


def text_encoder(W: Dict[str, Tensor], cfg, input_ids: Tensor) -> Tensor:
    """Qwen3Model.forward as the reference calls it (``conditioning_embed.py:71-74``: no
    attention mask ⇒ the default causal mask): embedding lookup, Qwen3 decoder layers
    (same structure as AceStepEncoderLayer) under a causal additive mask, final norm.
    Weights: Qwen3Model state-dict names."""
    h = F.embedding(input_ids, W["embed_tokens.weight"])
    S, dt = h.shape[1], h.dtype
    idx = torch.arange(S)
    mask = torch.full((1, 1, S, S), torch.finfo(dt).min, dtype=dt).masked_fill_(
        (idx[None, :] <= idx[:, None])[None, None], 0.0)
    cos, sin = rope_tables(S, cfg.head_dim, cfg.rope_theta, dt)
    cos, sin = cos.unsqueeze(1), sin.unsqueeze(1)
    for i in range(cfg.num_hidden_layers):
        h = encoder_layer(W, f"layers.{i}", cfg, h, mask, cos, sin)
    return rms_norm(h, W["norm.weight"], cfg.rms_norm_eps)
