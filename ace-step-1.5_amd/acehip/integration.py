"""Plug acehip into a running reference ``AceStepHandler`` (no caller edits).

Seams:
  * init   — ``_initialize_mlx_backends`` (``init_service_setup.py:116-148``) is
             where the reference converts weights for an alternative backend;
             :func:`install` does the same from ``handler.model`` /
             ``handler.vae`` state dicts.
  * DiT    — ``self.model.generate_audio(**generate_kwargs)``
             (``service_generate_execute.py:191,194``): replaced by
             :class:`~acehip.dit.AceStepDiTBackend.generate_audio` with the
             reference's own ``prepare_condition`` for the conditioning.
  * VAE    — ``handler.vae.decode(z).sample`` (``vae_decode_chunks.py:42,95``)
             and ``handler.vae.encode(x).latent_dist.sample()``
             (``vae_encode.py:65``): replaced by :class:`~acehip.vae.OobleckBackend`.

Failure policy: by default an acehip error propagates (the request fails
loudly, ``generate_music.py:181-190`` turns it into an error payload).  The
MLX precedent instead logs and falls back to the PyTorch path
(``service_generate_execute.py:189-191``); pass ``fallback=True`` to get that
behaviour — the fallback is the reference's own GPU path, never a CPU path.
"""
from __future__ import annotations

import logging
from typing import Optional

from .config import VAEConfig
from .dit import AceStepDiTBackend
from .vae import OobleckBackend

log = logging.getLogger("acehip")


def vae_from_diffusers(vae, max_seconds: float = 600.0, with_encoder: bool = True) -> OobleckBackend:
    """Build an OobleckBackend from a loaded diffusers ``AutoencoderOobleck``
    (precedent: ``acestep/models/mlx/vae_convert.py:37-132``)."""
    c = vae.config
    cfg = VAEConfig(encoder_hidden_size=c.encoder_hidden_size,
                    downsampling_ratios=list(c.downsampling_ratios),
                    channel_multiples=list(c.channel_multiples), decoder_channels=c.decoder_channels,
                    decoder_input_channels=c.decoder_input_channels, audio_channels=c.audio_channels)
    dev = next(vae.parameters()).device
    be = OobleckBackend(cfg, dev.index or 0, max_T=int(max_seconds * 48000 / cfg.hop_length) + 1,
                        with_encoder=with_encoder)
    be.load(vae.state_dict())
    return be


def install(handler, max_seconds: float = 600.0, max_batch: int = 8, fallback: bool = False,
            vae: bool = True) -> dict:
    """Swap the handler's DiT sampler and VAE for the acehip backends."""
    dit = AceStepDiTBackend.from_reference_model(handler.model, max_seconds=max_seconds,
                                                 max_batch=max_batch)
    orig_generate = handler.model.generate_audio

    def generate_audio(**kw):
        try:
            return dit.generate_audio(**kw)
        except Exception as e:  # pragma: no cover - exercised only with fallback=True
            if not fallback:
                raise
            log.warning("acehip generate_audio failed (%s); falling back to PyTorch", e)
            return orig_generate(**kw)

    handler.model.generate_audio = generate_audio
    out = {"dit": dit}
    if vae and getattr(handler, "vae", None) is not None:
        vb = vae_from_diffusers(handler.vae, max_seconds=max_seconds)
        orig_decode, orig_encode = handler.vae.decode, handler.vae.encode

        def decode(z, *a, **k):
            try:
                return vb.decode(z)
            except Exception as e:  # pragma: no cover
                if not fallback:
                    raise
                log.warning("acehip vae.decode failed (%s); falling back", e)
                return orig_decode(z, *a, **k)

        def encode(x, *a, **k):
            try:
                return vb.encode(x)
            except Exception as e:  # pragma: no cover
                if not fallback:
                    raise
                log.warning("acehip vae.encode failed (%s); falling back", e)
                return orig_encode(x, *a, **k)

        handler.vae.decode = decode
        handler.vae.encode = encode
        out["vae"] = vb
    return out
