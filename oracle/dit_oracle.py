"""CPU restatement of the ACE-Step 1.5 DiT decoder forward — TEST ORACLE ONLY.

Functional PyTorch-CPU code (no nn.Module) that reproduces, operation by
operation and in the caller's dtype, what ``AceStepDiTModel.forward`` computes
(reference ``acestep/models/base/modeling_acestep_v15_base.py``).  Each
function cites the reference lines it restates.  It is the checker the HIP
path is compared against and the ``cpu_baseline`` timed by ``bench.py``; the
product path never imports it.

Weights are a flat ``dict[str, Tensor]`` keyed by the reference state-dict
names *without* the ``decoder.`` prefix (SURVEY §8b weight contract).
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


def rms_norm(x: Tensor, w: Tensor, eps: float) -> Tensor:
    """Qwen3RMSNorm (transformers models/qwen3/modeling_qwen3.py:59-64):
    fp32 statistics, cast back to the input dtype, THEN the weight multiply."""
    dt = x.dtype
    h = x.to(torch.float32)
    h = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps)
    return w * h.to(dt)


def timestep_embedding(W: Dict[str, Tensor], prefix: str, t: Tensor,
                       n_freq: int = 256, scale: float = 1000.0) -> Tuple[Tensor, Tensor]:
    """TimestepEmbedding.forward (base:225-254).

    ``t*scale`` happens in t's dtype (bf16 rounds 0.75*1000 to 752 — the
    parity-critical detail of SURVEY §8a a7); the sinusoid is fp32."""
    ts = t * scale
    half = n_freq // 2
    freqs = torch.exp(-math.log(10000) * torch.arange(0, half, dtype=torch.float32) / half).to(t.device)
    args = ts[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    h = F.linear(emb.to(t.dtype), W[f"{prefix}.linear_1.weight"], W[f"{prefix}.linear_1.bias"])
    h = F.silu(h)
    temb = F.linear(h, W[f"{prefix}.linear_2.weight"], W[f"{prefix}.linear_2.bias"])
    proj = F.linear(F.silu(temb), W[f"{prefix}.time_proj.weight"], W[f"{prefix}.time_proj.bias"])
    return temb, proj.unflatten(1, (6, -1))


def rope_tables(S: int, head_dim: int, theta: float, dtype, device="cpu") -> Tuple[Tensor, Tensor]:
    """Qwen3RotaryEmbedding default init + forward (modeling_qwen3.py:116-137):
    fp32 inv_freq, positions 0..S-1, cat(freqs,freqs), cos/sin cast to dtype.

    The reference loader casts the whole model with ``.to(dtype)``
    (init_service_loader.py:81-89), which also casts the non-persistent
    ``inv_freq`` buffer: in bf16 mode the frequencies are bf16-rounded before
    the fp32 outer product."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float) / head_dim))
    inv = inv.to(dtype).float().to(device)
    pos = torch.arange(S, dtype=torch.float32, device=device)
    freqs = (inv[None, :, None] @ pos[None, None, :]).transpose(1, 2)   # [1,S,hd/2]
    emb = torch.cat((freqs, freqs), dim=-1)
    return emb.cos().to(dtype), emb.sin().to(dtype)


def _rotate_half(x: Tensor) -> Tensor:
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), dim=-1)


def additive_mask(S_q: int, S_k: int, dtype, window: Optional[int], device="cpu") -> Tensor:
    """create_4d_mask (base:56-135) for the decoder's bidirectional case with
    no padding mask (the decoder forces padding masks to None, base:1384-1385):
    0 where |i-j| <= window (or everywhere for full/cross), finfo.min elsewhere."""
    n = max(S_q, S_k)
    idx = torch.arange(n, device=device)
    valid = torch.ones(n, n, dtype=torch.bool, device=device)
    if window is not None:
        valid = (idx[:, None] - idx[None, :]).abs() <= window
    m = torch.full((1, 1, n, n), torch.finfo(dtype).min, dtype=dtype, device=device)
    m.masked_fill_(valid[None, None], 0.0)
    return m[:, :, :S_q, :S_k]


def attention(q: Tensor, k: Tensor, v: Tensor, mask: Tensor, scale: float,
              impl: str = "sdpa") -> Tensor:
    """transformers sdpa_attention_forward / eager_attention_forward as the
    decoder calls them: GQA via repeat_kv (a mask is always passed, so
    enable_gqa is not used), is_causal False, dropout 0."""
    n_rep = q.shape[1] // k.shape[1]
    if n_rep > 1:
        k = k.repeat_interleave(n_rep, dim=1)
        v = v.repeat_interleave(n_rep, dim=1)
    if impl == "sdpa":
        return F.scaled_dot_product_attention(q, k, v, attn_mask=mask, dropout_p=0.0,
                                              scale=scale, is_causal=False)
    # eager: fp32 softmax then cast (modeling_qwen3.py eager_attention_forward)
    s = torch.matmul(q, k.transpose(2, 3)) * scale + mask
    p = torch.softmax(s, dim=-1, dtype=torch.float32).to(q.dtype)
    return torch.matmul(p, v)


def cross_kv(W: Dict[str, Tensor], cfg, enc: Tensor) -> list:
    """condition_embedder (base:1359) + per-layer cross K/V computed once and
    cached (base:310-333): K = k_norm(k_proj(enc)), V = v_proj(enc)."""
    B, L, _ = enc.shape
    hd = cfg.head_dim
    e = F.linear(enc, W["condition_embedder.weight"], W["condition_embedder.bias"])
    out = []
    for i in range(cfg.num_hidden_layers):
        p = f"layers.{i}.cross_attn"
        k = rms_norm(F.linear(e, W[f"{p}.k_proj.weight"]).view(B, L, -1, hd),
                     W[f"{p}.k_norm.weight"], cfg.rms_norm_eps).transpose(1, 2)
        v = F.linear(e, W[f"{p}.v_proj.weight"]).view(B, L, -1, hd).transpose(1, 2)
        out.append((k, v))
    return out


def dit_forward(W: Dict[str, Tensor], cfg, xt: Tensor, t: Tensor, t_r: Tensor,
                enc: Tensor, ctx: Tensor, kv_cache: Optional[list] = None,
                attn_impl: str = "sdpa", return_hidden: bool = False) -> Tensor:
    """AceStepDiTModel.forward (base:1303-1507) + AceStepDiTLayer.forward
    (base:475-539) + AceStepAttention.forward (base:289-371).

    xt [B,T,64], t/t_r [B], enc [B,Lenc,D] (pre condition_embedder),
    ctx [B,T,128] → vt [B,T,64], all in xt's dtype."""
    dt = xt.dtype
    hd, eps = cfg.head_dim, cfg.rms_norm_eps
    scale = hd ** -0.5
    temb_t, proj_t = timestep_embedding(W, "time_embed", t)
    temb_r, proj_r = timestep_embedding(W, "time_embed_r", t - t_r)
    temb = temb_t + temb_r
    proj = proj_t + proj_r

    h = torch.cat([ctx, xt], dim=-1)
    T = h.shape[1]
    if T % cfg.patch_size:
        h = F.pad(h, (0, 0, 0, cfg.patch_size - T % cfg.patch_size))
    h = F.conv1d(h.transpose(1, 2), W["proj_in.1.weight"], W["proj_in.1.bias"],
                 stride=cfg.patch_size).transpose(1, 2)
    if kv_cache is None:
        kv_cache = cross_kv(W, cfg, enc)
    B, S, D = h.shape
    Lenc = kv_cache[0][0].shape[2]
    dev = xt.device      # the oracle also runs as torch-on-device for the full-length checks
    full_mask = additive_mask(S, S, dt, None, dev)
    band_mask = additive_mask(S, S, dt, cfg.sliding_window, dev)
    enc_mask = additive_mask(S, Lenc, dt, None, dev)
    cos, sin = rope_tables(S, hd, cfg.rope_theta, dt, dev)
    cos, sin = cos.unsqueeze(1), sin.unsqueeze(1)

    for i in range(cfg.num_hidden_layers):
        p = f"layers.{i}"
        sh, sc, g, csh, csc, cg = (W[f"{p}.scale_shift_table"] + proj).chunk(6, dim=1)
        # self-attention with AdaLN (base:499-511)
        x = (rms_norm(h, W[f"{p}.self_attn_norm.weight"], eps) * (1 + sc) + sh).type_as(h)
        a = f"{p}.self_attn"
        q = rms_norm(F.linear(x, W[f"{a}.q_proj.weight"]).view(B, S, -1, hd),
                     W[f"{a}.q_norm.weight"], eps).transpose(1, 2)
        k = rms_norm(F.linear(x, W[f"{a}.k_proj.weight"]).view(B, S, -1, hd),
                     W[f"{a}.k_norm.weight"], eps).transpose(1, 2)
        v = F.linear(x, W[f"{a}.v_proj.weight"]).view(B, S, -1, hd).transpose(1, 2)
        q = q * cos + _rotate_half(q) * sin
        k = k * cos + _rotate_half(k) * sin
        mask = band_mask if cfg.is_sliding(i) else full_mask
        o = attention(q, k, v, mask, scale, attn_impl).transpose(1, 2).reshape(B, S, -1)
        o = F.linear(o, W[f"{a}.o_proj.weight"])
        h = (h + o * g).type_as(h)
        # cross-attention, plain residual (base:513-526)
        x = rms_norm(h, W[f"{p}.cross_attn_norm.weight"], eps).type_as(h)
        c = f"{p}.cross_attn"
        q = rms_norm(F.linear(x, W[f"{c}.q_proj.weight"]).view(B, S, -1, hd),
                     W[f"{c}.q_norm.weight"], eps).transpose(1, 2)
        kc, vc = kv_cache[i]
        o = attention(q, kc, vc, enc_mask, scale, attn_impl).transpose(1, 2).reshape(B, S, -1)
        h = h + F.linear(o, W[f"{c}.o_proj.weight"])
        # SwiGLU MLP with AdaLN (base:528-533; Qwen3MLP)
        x = (rms_norm(h, W[f"{p}.mlp_norm.weight"], eps) * (1 + csc) + csh).type_as(h)
        m = f"{p}.mlp"
        ff = F.linear(F.silu(F.linear(x, W[f"{m}.gate_proj.weight"])) * F.linear(x, W[f"{m}.up_proj.weight"]),
                      W[f"{m}.down_proj.weight"])
        h = (h + ff * cg).type_as(h)

    if return_hidden:
        return h
    shift, sc = (W["scale_shift_table"] + temb.unsqueeze(1)).chunk(2, dim=1)
    h = (rms_norm(h, W["norm_out.weight"], eps) * (1 + sc) + shift).type_as(h)
    h = F.conv_transpose1d(h.transpose(1, 2), W["proj_out.1.weight"], W["proj_out.1.bias"],
                           stride=cfg.patch_size).transpose(1, 2)
    return h[:, :T]
