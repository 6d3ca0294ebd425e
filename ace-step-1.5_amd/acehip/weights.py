"""Weight-name contracts and synthetic (random-init) weights.

Name/shape contracts follow the reference state dicts:
DiT keys of ``AceStepDiTModel`` (reference ``modeling_acestep_v15_base.py``
:443-539 layers, :1240-1300 top level) and diffusers ``AutoencoderOobleck``
keys as mirrored by ``acestep/models/mlx/vae_model.py`` / ``vae_convert.py``.

Synthetic draw: every tensor from NumPy
``PCG64(base_seed ^ crc32(name))``.  ``mode="bench"`` is the §8d distribution
(linear N(0,0.02), biases 0, norms 1, Snake 0, weight_g = ||v||);
``mode="parity"`` perturbs biases/norm weights/Snake params/weight_g so that
parity tests exercise every term.  ``backend="torch"`` draws the same
distributions with a seeded device generator (fast path for the full-size
bench model; not bit-identical to the NumPy draw).
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, Tuple

import numpy as np
import torch

from .config import DiTConfig, VAEConfig

Shape = Tuple[int, ...]


def dit_weight_shapes(cfg: DiTConfig) -> Dict[str, Shape]:
    D, F_, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    qd, kvd = cfg.q_dim, cfg.kv_dim
    s: Dict[str, Shape] = {}
    for i in range(cfg.num_hidden_layers):
        p = f"layers.{i}"
        s[f"{p}.scale_shift_table"] = (1, 6, D)
        for n in ("self_attn_norm", "cross_attn_norm", "mlp_norm"):
            s[f"{p}.{n}.weight"] = (D,)
        for a in ("self_attn", "cross_attn"):
            s[f"{p}.{a}.q_proj.weight"] = (qd, D)
            s[f"{p}.{a}.k_proj.weight"] = (kvd, D)
            s[f"{p}.{a}.v_proj.weight"] = (kvd, D)
            s[f"{p}.{a}.o_proj.weight"] = (D, qd)
            s[f"{p}.{a}.q_norm.weight"] = (hd,)
            s[f"{p}.{a}.k_norm.weight"] = (hd,)
        s[f"{p}.mlp.gate_proj.weight"] = (F_, D)
        s[f"{p}.mlp.up_proj.weight"] = (F_, D)
        s[f"{p}.mlp.down_proj.weight"] = (D, F_)
    s["scale_shift_table"] = (1, 2, D)
    s["proj_in.1.weight"] = (D, cfg.in_channels, cfg.patch_size)
    s["proj_in.1.bias"] = (D,)
    for te in ("time_embed", "time_embed_r"):
        s[f"{te}.linear_1.weight"] = (D, 256)
        s[f"{te}.linear_1.bias"] = (D,)
        s[f"{te}.linear_2.weight"] = (D, D)
        s[f"{te}.linear_2.bias"] = (D,)
        s[f"{te}.time_proj.weight"] = (6 * D, D)
        s[f"{te}.time_proj.bias"] = (6 * D,)
    s["condition_embedder.weight"] = (D, D)
    s["condition_embedder.bias"] = (D,)
    s["norm_out.weight"] = (D,)
    s["proj_out.1.weight"] = (D, cfg.audio_acoustic_hidden_dim, cfg.patch_size)
    s["proj_out.1.bias"] = (cfg.audio_acoustic_hidden_dim,)
    return s


def encoder_stack_shapes(cfg: DiTConfig, prefix: str, n_layers: int, in_dim: int, embed_bias: bool,
                         out_dim: int = 0) -> Dict[str, Shape]:
    """One AceStepEncoderLayer stack (base:374-440) with embed_tokens / norm /
    optional proj_out, module-local names under ``prefix``."""
    D, F_, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    qd, kvd = cfg.q_dim, cfg.kv_dim
    s: Dict[str, Shape] = {f"{prefix}.embed_tokens.weight": (D, in_dim)}
    if embed_bias:
        s[f"{prefix}.embed_tokens.bias"] = (D,)
    for i in range(n_layers):
        p = f"{prefix}.layers.{i}"
        s[f"{p}.input_layernorm.weight"] = (D,)
        s[f"{p}.post_attention_layernorm.weight"] = (D,)
        s[f"{p}.self_attn.q_proj.weight"] = (qd, D)
        s[f"{p}.self_attn.k_proj.weight"] = (kvd, D)
        s[f"{p}.self_attn.v_proj.weight"] = (kvd, D)
        s[f"{p}.self_attn.o_proj.weight"] = (D, qd)
        s[f"{p}.self_attn.q_norm.weight"] = (hd,)
        s[f"{p}.self_attn.k_norm.weight"] = (hd,)
        s[f"{p}.mlp.gate_proj.weight"] = (F_, D)
        s[f"{p}.mlp.up_proj.weight"] = (F_, D)
        s[f"{p}.mlp.down_proj.weight"] = (D, F_)
    s[f"{prefix}.norm.weight"] = (D,)
    if out_dim:
        s[f"{prefix}.proj_out.weight"] = (out_dim, D)
        s[f"{prefix}.proj_out.bias"] = (out_dim,)
    return s


def condenc_weight_shapes(cfg: DiTConfig) -> Dict[str, Shape]:
    """AceStepConditionEncoder (base:1517-1525) module-local names: text_projector
    (no bias), lyric_encoder (embed with bias), timbre_encoder (embed with bias,
    special_token unused at inference, base:1087)."""
    s: Dict[str, Shape] = {"text_projector.weight": (cfg.hidden_size, cfg.text_hidden_dim)}
    s.update(encoder_stack_shapes(cfg, "lyric_encoder", cfg.num_lyric_encoder_hidden_layers,
                                  cfg.text_hidden_dim, True))
    s.update(encoder_stack_shapes(cfg, "timbre_encoder", cfg.num_timbre_encoder_hidden_layers,
                                  cfg.timbre_hidden_dim, True))
    s["timbre_encoder.special_token"] = (1, 1, cfg.hidden_size)
    return s


def tokenizer_weight_shapes(cfg: DiTConfig) -> Dict[str, Shape]:
    """AceStepAudioTokenizer (base:1189-1203) under ``tokenizer.`` and
    AudioTokenDetokenizer (base:870-886) under ``detokenizer.``; the quantizer is
    ResidualFSQ(dim=fsq_dim, levels [8,8,8,5,5,5]) → project_in / project_out."""
    D, nl = cfg.hidden_size, 6
    s: Dict[str, Shape] = {"tokenizer.audio_acoustic_proj.weight": (D, cfg.audio_acoustic_hidden_dim),
                           "tokenizer.audio_acoustic_proj.bias": (D,)}
    s.update(encoder_stack_shapes(cfg, "tokenizer.attention_pooler", cfg.num_attention_pooler_hidden_layers, D, True))
    s["tokenizer.attention_pooler.special_token"] = (1, 1, D)
    s["tokenizer.quantizer.project_in.weight"] = (nl, D)
    s["tokenizer.quantizer.project_in.bias"] = (nl,)
    s["tokenizer.quantizer.project_out.weight"] = (D, nl)
    s["tokenizer.quantizer.project_out.bias"] = (D,)
    s.update(encoder_stack_shapes(cfg, "detokenizer", cfg.num_attention_pooler_hidden_layers, D, True,
                                  out_dim=cfg.audio_acoustic_hidden_dim))
    s["detokenizer.special_tokens"] = (1, cfg.pool_window_size, D)
    return s


def text_encoder_shapes(cfg: DiTConfig, vocab: int) -> Dict[str, Shape]:
    """Qwen3Model (the Qwen3-Embedding-0.6B text encoder) state-dict names: embed_tokens
    (an nn.Embedding table), the decoder layers, the final norm."""
    s: Dict[str, Shape] = {"embed_tokens.weight": (vocab, cfg.hidden_size)}
    for k, v in encoder_stack_shapes(cfg, "_", cfg.num_hidden_layers, 0, False).items():
        if not k.startswith("_.embed_tokens"):
            s[k[2:]] = v
    return s


def synth_text_encoder_weights(cfg: DiTConfig, vocab: int, seed: int = 0, mode: str = "bench", **kw):
    return synth_weights(text_encoder_shapes(cfg, vocab), seed, mode, **kw)


def synth_tokenizer_weights(cfg: DiTConfig, seed: int = 0, mode: str = "bench", **kw):
    return synth_weights(tokenizer_weight_shapes(cfg), seed, mode, **kw)


def synth_condenc_weights(cfg: DiTConfig, seed: int = 0, mode: str = "bench", **kw):
    return synth_weights(condenc_weight_shapes(cfg), seed, mode, **kw)


def vae_weight_shapes(cfg: VAEConfig, with_encoder: bool = True) -> Dict[str, Shape]:
    s: Dict[str, Shape] = {}

    def conv(name, cout, cin, k, bias=True, transposed=False):
        shape = (cin, cout, k) if transposed else (cout, cin, k)
        s[name + ".weight_v"] = shape
        s[name + ".weight_g"] = (shape[0], 1, 1)
        if bias:
            s[name + ".bias"] = (cout,)

    def snk(name, c):
        s[name + ".alpha"] = (1, c, 1)
        s[name + ".beta"] = (1, c, 1)

    def res(p, c):
        for n in (1, 2, 3):
            snk(f"{p}.res_unit{n}.snake1", c)
            conv(f"{p}.res_unit{n}.conv1", c, c, 7)
            snk(f"{p}.res_unit{n}.snake2", c)
            conv(f"{p}.res_unit{n}.conv2", c, c, 1)

    blocks = cfg.decoder_block_channels()
    conv("decoder.conv1", blocks[0][0], cfg.decoder_input_channels, 7)
    for j, (cin, cout, st) in enumerate(blocks):
        p = f"decoder.block.{j}"
        snk(p + ".snake1", cin)
        conv(p + ".conv_t1", cout, cin, 2 * st, transposed=True)
        res(p, cout)
    snk("decoder.snake1", cfg.decoder_channels)
    conv("decoder.conv2", cfg.audio_channels, cfg.decoder_channels, 7, bias=False)
    if with_encoder:
        eb = cfg.encoder_block_channels()
        conv("encoder.conv1", cfg.encoder_hidden_size, cfg.audio_channels, 7)
        for j, (cin, cout, st) in enumerate(eb):
            p = f"encoder.block.{j}"
            res(p, cin)
            snk(p + ".snake1", cin)
            conv(p + ".conv1", cout, cin, 2 * st)
        snk("encoder.snake1", eb[-1][1])
        conv("encoder.conv2", cfg.encoder_hidden_size, eb[-1][1], 3)
    return s


def _kind(name: str) -> str:
    if name.endswith("scale_shift_table"):
        return "sst"
    if name.endswith("null_condition_emb"):
        return "unit"
    if name.endswith(".bias"):
        return "bias"
    if name.endswith((".alpha", ".beta")):
        return "snake"
    if name.endswith(".weight_g"):
        return "g"
    if name.endswith("norm.weight") or name.endswith("_norm.weight") or name == "norm_out.weight":
        return "norm"
    return "w"


def _draw(rng: np.random.Generator, name: str, shape: Shape, mode: str) -> np.ndarray:
    k = _kind(name)
    if k == "w":
        return rng.normal(0.0, 0.02, size=shape).astype(np.float32)
    if k == "sst":
        return (rng.normal(0.0, 1.0, size=shape) / math.sqrt(shape[-1])).astype(np.float32)
    if k == "unit":
        return rng.normal(0.0, 1.0, size=shape).astype(np.float32)
    if mode == "bench":
        return (np.ones(shape) if k == "norm" else np.zeros(shape)).astype(np.float32)
    if k == "norm":
        return (1.0 + rng.normal(0.0, 0.1, size=shape)).astype(np.float32)
    if k == "bias":
        return rng.normal(0.0, 0.02, size=shape).astype(np.float32)
    if k == "snake":
        return rng.normal(0.0, 0.2, size=shape).astype(np.float32)
    return np.zeros(shape, np.float32)  # weight_g placeholder, set from ||v|| below


def synth_weights(shapes: Dict[str, Shape], seed: int = 0, mode: str = "bench",
                  dtype=torch.float32, device="cpu", backend: str = "numpy",
                  workers: int = 1) -> Dict[str, torch.Tensor]:
    """``workers`` > 1 draws the NumPy tensors on a thread pool (each tensor has its own
    PCG64 stream, so the result does not depend on the worker count; NumPy releases the
    GIL inside the draw) — the full 24-layer DiT is 1.58 G values, ≈ 40 s on one thread."""
    out: Dict[str, torch.Tensor] = {}
    if backend == "numpy" and workers > 1:
        from concurrent.futures import ThreadPoolExecutor

        def one(item):
            name, shape = item
            s = (seed ^ zlib.crc32(name.encode())) & 0xFFFFFFFF
            return name, _draw(np.random.Generator(np.random.PCG64(s)), name, shape, mode)
        with ThreadPoolExecutor(workers) as ex:
            for name, arr in ex.map(one, shapes.items()):
                out[name] = torch.from_numpy(arr).to(device=device, dtype=dtype)
    for name, shape in shapes.items():
        if name in out:
            continue
        s = (seed ^ zlib.crc32(name.encode())) & 0xFFFFFFFF
        if backend == "numpy":
            arr = _draw(np.random.Generator(np.random.PCG64(s)), name, shape, mode)
            out[name] = torch.from_numpy(arr).to(device=device, dtype=dtype)
        else:
            g = torch.Generator(device=device).manual_seed(s)
            k = _kind(name)
            if k == "w":
                t = torch.randn(shape, generator=g, device=device, dtype=torch.float32) * 0.02
            elif k == "sst":
                t = torch.randn(shape, generator=g, device=device) / math.sqrt(shape[-1])
            elif k == "unit":
                t = torch.randn(shape, generator=g, device=device)
            elif k == "norm" and mode == "bench":
                t = torch.ones(shape, device=device)
            elif mode == "bench" or k == "g":
                t = torch.zeros(shape, device=device)
            elif k == "norm":
                t = 1.0 + 0.1 * torch.randn(shape, generator=g, device=device)
            elif k == "bias":
                t = 0.02 * torch.randn(shape, generator=g, device=device)
            else:
                t = 0.2 * torch.randn(shape, generator=g, device=device)
            out[name] = t.to(dtype)
    # weight_g = ||v|| (identity weight-norm) in bench mode, a random gain in parity mode
    for name in shapes:
        if name.endswith(".weight_g"):
            v = out[name[:-2] + "_v"].float()
            n = v.reshape(v.shape[0], -1).norm(dim=1).reshape(shapes[name])
            if mode == "parity":
                s = (seed ^ zlib.crc32(name.encode())) & 0xFFFFFFFF
                gain = np.random.Generator(np.random.PCG64(s)).uniform(0.5, 1.5, size=shapes[name])
                n = n * torch.from_numpy(gain.astype(np.float32)).to(n.device)
            out[name] = n.to(dtype)
    return out


def synth_dit_weights(cfg: DiTConfig, seed: int = 0, mode: str = "bench", **kw):
    w = synth_weights(dit_weight_shapes(cfg), seed, mode, **kw)
    return w


def synth_null_condition(cfg: DiTConfig, seed: int = 0, **kw) -> torch.Tensor:
    """``null_condition_emb`` (1,1,D) N(0,1) (base:1575)."""
    return synth_weights({"null_condition_emb": (1, 1, cfg.hidden_size)}, seed, "bench", **kw)[
        "null_condition_emb"]


def synth_vae_weights(cfg: VAEConfig, seed: int = 0, mode: str = "bench", with_encoder=True, **kw):
    return synth_weights(vae_weight_shapes(cfg, with_encoder), seed, mode, **kw)
