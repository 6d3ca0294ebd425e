"""CPU restatement of the Oobleck VAE (diffusers ``AutoencoderOobleck``) — TEST ORACLE ONLY.

**parity unpinned**: the reference delegates this arithmetic to the
third-party ``diffusers`` package (version unpinned in the reference's
``requirements.txt``; not installed in this image) and no reference test pins
its numerics.  This restatement follows the reference's own structural spec of
that model, ``acestep/models/mlx/vae_model.py:24-336`` (Snake1d, residual
units, encoder/decoder blocks) and the weight-norm fusion of
``acestep/models/mlx/vae_convert.py:18-34`` (``w = g * v / ||v||`` with the
norm over every dim except dim 0 — the *input* channel for ConvTranspose1d).
Layout is channels-first ``[B, C, L]`` like diffusers.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


def fuse_weight_norm(g: Tensor, v: Tensor) -> Tensor:
    """torch weight_norm(dim=0): v * g / ||v|| (norm over all dims but 0)."""
    n = v.reshape(v.shape[0], -1).norm(dim=1).reshape(g.shape)
    return v * (g / n)


def _w(W: Dict[str, Tensor], name: str) -> Tensor:
    if name + ".weight" in W:
        return W[name + ".weight"]
    if name + ".weight_g" in W:
        return fuse_weight_norm(W[name + ".weight_g"], W[name + ".weight_v"])
    return fuse_weight_norm(W[name + ".parametrizations.weight.original0"],
                            W[name + ".parametrizations.weight.original1"])


def snake(x: Tensor, alpha: Tensor, beta: Tensor) -> Tensor:
    """Snake1d with logscale (vae_model.py:38-55): x + 1/(e^β+1e-9)·sin(e^α·x)²."""
    a = torch.exp(alpha).reshape(1, -1, 1)
    b = torch.exp(beta).reshape(1, -1, 1)
    return x + (b + 1e-9).reciprocal() * torch.sin(a * x).pow(2)


def _snake(W, prefix, x):
    return snake(x, W[prefix + ".alpha"], W[prefix + ".beta"])


def _res_unit(W, p, x, dilation):
    """OobleckResidualUnit (vae_model.py:62-87)."""
    y = F.conv1d(_snake(W, p + ".snake1", x), _w(W, p + ".conv1"), W[p + ".conv1.bias"],
                 dilation=dilation, padding=3 * dilation)
    y = F.conv1d(_snake(W, p + ".snake2", y), _w(W, p + ".conv2"), W[p + ".conv2.bias"])
    return x + y


def decode(W: Dict[str, Tensor], cfg, z: Tensor) -> Tensor:
    """OobleckDecoder (vae_model.py:190-230 + blocks :119-142): z [B,64,T] → [B,2,T·hop]."""
    x = F.conv1d(z, _w(W, "decoder.conv1"), W["decoder.conv1.bias"], padding=3)
    for j, (_cin, _cout, s) in enumerate(cfg.decoder_block_channels()):
        p = f"decoder.block.{j}"
        x = _snake(W, p + ".snake1", x)
        x = F.conv_transpose1d(x, _w(W, p + ".conv_t1"), W[p + ".conv_t1.bias"],
                               stride=s, padding=math.ceil(s / 2))
        for n, d in ((1, 1), (2, 3), (3, 9)):
            x = _res_unit(W, f"{p}.res_unit{n}", x, d)
    x = _snake(W, "decoder.snake1", x)
    return F.conv1d(x, _w(W, "decoder.conv2"), None, padding=3)


def encode_moments(W: Dict[str, Tensor], cfg, wav: Tensor) -> Tensor:
    """OobleckEncoder (vae_model.py:149-187 + blocks :94-116): [B,2,N] → [B,128,N/hop]."""
    x = F.conv1d(wav, _w(W, "encoder.conv1"), W["encoder.conv1.bias"], padding=3)
    for j, (_cin, _cout, s) in enumerate(cfg.encoder_block_channels()):
        p = f"encoder.block.{j}"
        for n, d in ((1, 1), (2, 3), (3, 9)):
            x = _res_unit(W, f"{p}.res_unit{n}", x, d)
        x = _snake(W, p + ".snake1", x)
        x = F.conv1d(x, _w(W, p + ".conv1"), W[p + ".conv1.bias"], stride=s,
                     padding=math.ceil(s / 2))
    x = _snake(W, "encoder.snake1", x)
    return F.conv1d(x, _w(W, "encoder.conv2"), W["encoder.conv2.bias"], padding=1)


def encode_sample(W, cfg, wav: Tensor, noise: Optional[Tensor] = None) -> Tensor:
    """latent_dist.sample() (vae_model.py:285-304): mean + (softplus(scale)+1e-4)·ε."""
    h = encode_moments(W, cfg, wav)
    mean, sc = h.chunk(2, dim=1)
    if noise is None:
        return mean
    std = F.softplus(sc) + 1e-4
    return mean + std * noise


# ---------------------------------------------------------------------------------------------
# bf16-storage variant (test oracle for the HIP path at the reference's GPU precision): every
# activation is STORED in bf16 between ops — as the reference's bf16 VAE on the GPU stores it —
# while each conv / Snake / residual computes in fp32 (MIOpen / rocBLAS bf16 convolutions
# accumulate in fp32 and round once).  Weights are the weight-norm fusion rounded to bf16.
# Runs as torch on any device (the full-length GPU tests run it on the GPU in fp32 arithmetic).
def _rb(x: Tensor) -> Tensor:
    return x.to(torch.bfloat16).to(torch.float32)


def _wb(W: Dict[str, Tensor], name: str) -> Tensor:
    Wf = {k: v.float() for k, v in W.items() if k.startswith(name + ".")}
    return _rb(_w(Wf, name))


def _bb(W: Dict[str, Tensor], name: str) -> Optional[Tensor]:
    return _rb(W[name].float()) if name in W else None


def _snake_b(W, prefix, x):
    return _rb(snake(x, W[prefix + ".alpha"].float(), W[prefix + ".beta"].float()))


def _res_unit_b(W, p, x, dilation):
    y = _rb(F.conv1d(_snake_b(W, p + ".snake1", x), _wb(W, p + ".conv1"), _bb(W, p + ".conv1.bias"),
                     dilation=dilation, padding=3 * dilation))
    y = _rb(F.conv1d(_snake_b(W, p + ".snake2", y), _wb(W, p + ".conv2"), _bb(W, p + ".conv2.bias")))
    return _rb(x + y)


def decode_bf16_storage(W: Dict[str, Tensor], cfg, z: Tensor) -> Tensor:
    """``decode`` with bf16 activations between ops and fp32 math inside each (see above)."""
    x = _rb(F.conv1d(_rb(z.float()), _wb(W, "decoder.conv1"), _bb(W, "decoder.conv1.bias"), padding=3))
    for j, (_cin, _cout, s) in enumerate(cfg.decoder_block_channels()):
        p = f"decoder.block.{j}"
        x = _snake_b(W, p + ".snake1", x)
        x = _rb(F.conv_transpose1d(x, _wb(W, p + ".conv_t1"), _bb(W, p + ".conv_t1.bias"),
                                   stride=s, padding=math.ceil(s / 2)))
        for n, d in ((1, 1), (2, 3), (3, 9)):
            x = _res_unit_b(W, f"{p}.res_unit{n}", x, d)
    x = _snake_b(W, "decoder.snake1", x)
    # the bf16 VAE's decode(z).sample is bf16 (upcast later by the handler, generate_music_decode.py:188)
    return _rb(F.conv1d(x, _wb(W, "decoder.conv2"), None, padding=3))


def encode_mean_bf16_storage(W: Dict[str, Tensor], cfg, wav: Tensor) -> Tensor:
    """``encode_sample(noise=None)`` (the mean) with bf16 activations between ops."""
    x = _rb(F.conv1d(_rb(wav.float()), _wb(W, "encoder.conv1"), _bb(W, "encoder.conv1.bias"), padding=3))
    for j, (_cin, _cout, s) in enumerate(cfg.encoder_block_channels()):
        p = f"encoder.block.{j}"
        for n, d in ((1, 1), (2, 3), (3, 9)):
            x = _res_unit_b(W, f"{p}.res_unit{n}", x, d)
        x = _snake_b(W, p + ".snake1", x)
        x = _rb(F.conv1d(x, _wb(W, p + ".conv1"), _bb(W, p + ".conv1.bias"), stride=s, padding=math.ceil(s / 2)))
    x = _snake_b(W, "encoder.snake1", x)
    h = F.conv1d(x, _wb(W, "encoder.conv2"), _bb(W, "encoder.conv2.bias"), padding=1)
    return h.chunk(2, dim=1)[0]
