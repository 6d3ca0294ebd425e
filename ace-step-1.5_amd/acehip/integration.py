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
             (``vae_encode.py:65``): replaced by :class:`~acehip.vae.OobleckBackend`;
             ``handler.tiled_encode`` (``vae_encode.py:15-82``: 30 s chunks, 2 s
             overlap, per-chunk host offload) becomes ONE untiled encode;
             ``handler.tiled_decode`` (``vae_decode.py:16-85``, called at
             ``generate_music_decode.py:164``) becomes ONE untiled decode of the
             whole batch — the reference's overlap-discard windows (1.6x the useful
             frames at 240 s) are redundant because the decoder's receptive field
             (-8.2/+9.2 frames) is inside the 64-frame overlap (tiled == untiled,
             tests/test_gpu_long.py).

  * cond   — ``prepare_condition`` (``base:1607-1652``, called from
             ``generate_audio`` ``base:1820``): replaced by
             :class:`~acehip.condition.HipPrepareCondition` (text projector, lyric
             and timbre encoders, and for covers the audio tokenizer (pooler + FSQ)
             and detokenizer, all on libacehip).
  * LoRA   — ``add_lora`` / ``remove_lora`` / ``unload_lora`` / ``set_lora_scale`` /
             ``set_use_lora`` / ``set_active_lora_adapter`` (``handler/lora/lifecycle.py:164-420``,
             ``lora/controls.py:12-157``) change the decoder's effective weights;
             :func:`install` wraps them so the merged weights are re-packed into the
             handle afterwards (:func:`refresh_decoder_weights`).

Failure policy: by default an acehip error propagates (the request fails
loudly, ``generate_music.py:181-190`` turns it into an error payload).  The
MLX precedent instead logs and falls back to the PyTorch path
(``service_generate_execute.py:189-191``); pass ``fallback=True`` to get that
behaviour — the fallback is the reference's own GPU path, never a CPU path.
"""
from __future__ import annotations

import logging
from typing import Optional

import torch

from .condition import AudioDetokenizer, AudioTokenizer, ConditionEncoder, HipPrepareCondition, TextEncoder
from .config import VAEConfig
from .dit import AceStepDiTBackend
from .vae import OobleckBackend

log = logging.getLogger("acehip")


def vae_from_diffusers(vae, max_seconds: float = 600.0, with_encoder: bool = True,
                       max_batch: int = 8) -> OobleckBackend:
    """Build an OobleckBackend from a loaded diffusers ``AutoencoderOobleck``
    (precedent: ``acestep/models/mlx/vae_convert.py:37-132``)."""
    c = vae.config
    cfg = VAEConfig(encoder_hidden_size=c.encoder_hidden_size,
                    downsampling_ratios=list(c.downsampling_ratios),
                    channel_multiples=list(c.channel_multiples), decoder_channels=c.decoder_channels,
                    decoder_input_channels=c.decoder_input_channels, audio_channels=c.audio_channels)
    dev = next(vae.parameters()).device
    be = OobleckBackend(cfg, dev.index or 0, max_T=int(max_seconds * 48000 / cfg.hop_length) + 1,
                        max_B=max_batch, with_encoder=with_encoder)
    be.load(vae.state_dict())
    return be


def merged_decoder_state_dict(decoder) -> dict:
    """Effective (adapter-merged) decoder weights under the plain HF names.

    Works on a bare ``AceStepDiTModel`` and on a PEFT-wrapped one (``PeftModel``
    / LoRA layers with ``base_layer`` + ``get_delta_weight``, as created by
    ``lifecycle.py:249-258``; LyCORIS LoKr modules expose the same two): every
    adapted Linear becomes ``base.weight + Σ_active get_delta_weight(a)`` unless
    the adapters are disabled or already merged; PEFT's name decorations
    (``base_model.model.``, ``.base_layer``) are stripped."""
    out = {}
    with torch.no_grad():
        for name, mod in decoder.named_modules():
            base = getattr(mod, "base_layer", None)
            if base is None or not hasattr(mod, "get_delta_weight"):
                continue
            w = base.weight.detach().float().clone()
            if not getattr(mod, "disable_adapters", False) and not getattr(mod, "merged", False):
                act = getattr(mod, "active_adapters", None) or []
                for a in ([act] if isinstance(act, str) else act):
                    try:
                        w += mod.get_delta_weight(a).float()
                    except KeyError:      # adapter not present on this layer
                        pass
            out[name + ".weight"] = w
            if getattr(base, "bias", None) is not None:
                out[name + ".bias"] = base.bias.detach()
        for k, v in decoder.state_dict().items():
            if ".base_layer." in k or "lora_" in k or "lokr_" in k or ".hada_" in k:
                continue
            out.setdefault(k, v)
    clean = {}
    for k, v in out.items():
        if k.startswith("base_model.model."):
            k = k[len("base_model.model."):]
        clean[k.replace(".base_layer", "")] = v
    return clean


def refresh_decoder_weights(dit: AceStepDiTBackend, decoder) -> None:
    """Re-pack the decoder's current effective weights into the DiT handle
    (§8f row 3: LoRA add/remove/scale changes)."""
    dit.rt.load(merged_decoder_state_dict(decoder))


_LORA_METHODS = ("add_lora", "load_lora", "add_voice_lora", "remove_lora", "unload_lora", "set_lora_scale",
                 "set_use_lora", "set_active_lora_adapter")


def install(handler, max_seconds: float = 600.0, max_batch: int = 8, fallback: bool = False,
            vae: bool = True, condition: bool = True, text_encoder: bool = True) -> dict:
    """Swap the handler's DiT sampler, VAE and (Qwen3) text encoder for the acehip backends."""
    dit = AceStepDiTBackend.from_reference_model(handler.model, max_seconds=max_seconds,
                                                 max_batch=max_batch)
    if condition:
        ce = ConditionEncoder.from_reference_model(handler.model, max_batch=max_batch)
        tok = det = None
        m = handler.model
        if getattr(m, "tokenizer", None) is not None and getattr(m, "detokenizer", None) is not None:
            dev = ce.device.index or 0
            patches = int(max_seconds * 25) // ce.cfg.pool_window_size + 1
            tok = AudioTokenizer(ce.cfg, dev, max_patches=max_batch * patches)
            tok.load({"tokenizer." + k: v for k, v in m.tokenizer.state_dict().items()})
            det = AudioDetokenizer(ce.cfg, dev, max_patches=max_batch * patches)
            det.load({"detokenizer." + k: v for k, v in m.detokenizer.state_dict().items()})
        hip_prep = HipPrepareCondition(ce, fallback=m.prepare_condition, tokenizer=tok, detokenizer=det)
        # the handler calls prepare_condition itself (service_generate_execute.py:123-142) and then
        # generate_audio calls it again on the same payload (base:1820): the handler's call records
        # its outputs, generate_audio's consumes them — one encoder pass per request
        dit.prepare_condition = hip_prep.consume
        m.prepare_condition = hip_prep.record
        out_prep = hip_prep
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
    if condition:
        out["prepare_condition"] = out_prep

    # LoRA lifecycle: after any adapter change re-pack the merged decoder weights
    for meth in _LORA_METHODS:
        orig = getattr(handler, meth, None)
        if orig is None:
            continue

        def wrapped(*a, _orig=orig, **k):
            res = _orig(*a, **k)
            refresh_decoder_weights(dit, handler.model.decoder)
            return res
        setattr(handler, meth, wrapped)
    if text_encoder and getattr(handler, "text_encoder", None) is not None:
        # infer_text_embeddings / infer_lyric_embeddings (conditioning_embed.py:71-79)
        te = TextEncoder.from_reference_model(handler.text_encoder, device=dit.rt.device.index or 0,
                                              max_batch=max_batch)
        handler.text_encoder = te
        out["text_encoder"] = te
    if vae and getattr(handler, "vae", None) is not None:
        vb = vae_from_diffusers(handler.vae, max_seconds=max_seconds, max_batch=max_batch)
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
        orig_tiled = getattr(handler, "tiled_decode", None)

        def tiled_decode(latents, chunk_size=None, overlap=64, offload_wav_to_cpu=None):
            # vae_decode.py:16-85 contract: [B, 64, T] -> [B, 2, T*hop]; untiled here.
            # None resolves through the handler's policy as the reference does (:53-54)
            if offload_wav_to_cpu is None and hasattr(handler, "_should_offload_wav_to_cpu"):
                offload_wav_to_cpu = bool(handler._should_offload_wav_to_cpu())
            try:
                return vb.tiled_decode(latents, chunk_size, overlap, offload_wav_to_cpu)
            except Exception as e:  # pragma: no cover
                if not fallback or orig_tiled is None:
                    raise
                log.warning("acehip tiled_decode failed (%s); falling back", e)
                return orig_tiled(latents, chunk_size=chunk_size, overlap=overlap,
                                  offload_wav_to_cpu=offload_wav_to_cpu)
        handler.tiled_decode = tiled_decode
        orig_tiled_enc = getattr(handler, "tiled_encode", None)

        def tiled_encode(audio, chunk_size=None, overlap=None, offload_latent_to_cpu=True):
            # vae_encode.py:15-82 contract (batch_prep.py:70, conditioning_embed.py:58):
            # ONE untiled encode instead of the 30 s chunk loop
            try:
                return vb.tiled_encode(audio, chunk_size, overlap, offload_latent_to_cpu)
            except Exception as e:  # pragma: no cover
                if not fallback or orig_tiled_enc is None:
                    raise
                log.warning("acehip tiled_encode failed (%s); falling back", e)
                return orig_tiled_enc(audio, chunk_size=chunk_size, overlap=overlap,
                                      offload_latent_to_cpu=offload_latent_to_cpu)
        handler.tiled_encode = tiled_encode
        out["vae"] = vb
    return out


def hip_normalize_audio(audio_data: torch.Tensor, target_db: float = -1.0) -> torch.Tensor:
    """``normalize_audio`` (acestep/audio_utils.py:24-62) for device tensors: same
    contract (returns a new tensor; silence returned unchanged) on the fused HIP
    pass.  A caller that normalizes while the audio is still on the GPU (before the
    payload's host copy) can bind it in place of the CPU pass at inference.py:679."""
    if not (isinstance(audio_data, torch.Tensor) and audio_data.is_cuda):
        raise TypeError("hip_normalize_audio: a GPU tensor is required (no CPU path)")
    x = audio_data.detach().float().contiguous().clone().reshape(1, -1)
    if x.shape[1] % 4:
        raise ValueError("hip_normalize_audio: sample count must be a multiple of 4")
    peak = torch.empty(1, device=x.device, dtype=torch.float32)
    from ._ffi import check, lib, ptr, stream_ptr
    target = float(torch.tensor(10 ** (target_db / 20.0), dtype=torch.float32))
    if target_db > 0.0:
        raise ValueError("hip_normalize_audio: target_db must be <= 0 (inference.py:674)")
    # guard off: normalize_audio alone scales a peak above 1 in one multiply
    check(lib().acehip_wav_postprocess(ptr(x), 1, x.shape[1], ptr(peak), 0, target, stream_ptr()), "wav_normalize")
    return x.reshape(audio_data.shape).to(audio_data.dtype)
