"""Oobleck VAE backend: the ``vae.decode(z).sample`` / ``tiled_decode`` /
``vae.encode(x).latent_dist.sample()`` seams of the reference handler
(``acestep/core/generation/handler/vae_decode_chunks.py:42,95,119,147``,
``vae_decode.py:16-85``, ``vae_encode.py:65``) on libacehip's implicit-GEMM
HIP kernels.  No CPU fallback: the library must load.
"""
from __future__ import annotations

import os

from types import SimpleNamespace
from typing import Dict, Optional

import torch

from . import _ffi
from ._ffi import ACEHIP_BF16, ACEHIP_F32, check, lib, ptr, shape_arg, stream_ptr
from .config import VAEConfig


class OobleckBackend:
    def __init__(self, cfg: VAEConfig, device=0, max_T: int = 15000, max_B: int = 1,
                 with_encoder: bool = True):
        self.cfg = cfg
        self.device = torch.device("cuda", device if isinstance(device, int) else device.index or 0)
        self.max_T = max_T
        c = _ffi.VAECfg()
        c.encoder_hidden = cfg.encoder_hidden_size
        c.decoder_channels = cfg.decoder_channels
        c.latent_channels = cfg.decoder_input_channels
        c.audio_channels = cfg.audio_channels
        c.n_blocks = len(cfg.downsampling_ratios)
        for i, r in enumerate(cfg.downsampling_ratios):
            c.ratios[i] = r
        for i, m in enumerate(cfg.channel_multiples):
            c.multiples[i] = m
        c.max_T, c.max_B, c.with_encoder = max_T, max_B, 1 if with_encoder else 0
        self.with_encoder = with_encoder
        h = _ffi.c_void_p()
        check(lib().acehip_vae_create(self.device.index, _ffi.ctypes.byref(c), _ffi.ctypes.byref(h)),
              "vae_create")
        self.h = h
        self.hop = cfg.hop_length
        self.dtype = torch.bfloat16

    def load(self, weights: Dict[str, torch.Tensor]):
        """diffusers state-dict names (weight_g/weight_v or parametrizations.*)."""
        for k, v in weights.items():
            if k.startswith("encoder.") and not self.with_encoder:
                continue
            t = v.detach().contiguous()
            if t.dtype not in (torch.float32, torch.bfloat16):
                t = t.float()
            dt = ACEHIP_F32 if t.dtype == torch.float32 else ACEHIP_BF16
            check(lib().acehip_vae_set_weight(self.h, k.encode(), ptr(t), dt, t.dim(),
                                              shape_arg(tuple(t.shape)), 1 if t.is_cuda else 0),
                  f"vae_set_weight({k})")
        check(lib().acehip_vae_finalize(self.h), "vae_finalize")

    # ----------------------------------------------------------------- API --
    def decode_tensor(self, z: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """z [B, 64, T] → fp32 audio [B, 2, T·hop] (untiled)."""
        z = z.to(device=self.device, dtype=torch.bfloat16).contiguous()
        B, C, T = z.shape
        if out is None:
            out = torch.empty(B, self.cfg.audio_channels, T * self.hop, device=self.device,
                              dtype=torch.float32)
        check(lib().acehip_vae_decode(self.h, ptr(z), B, T, ptr(out), stream_ptr()), "vae_decode")
        return out

    @staticmethod
    def peak_normalize_(wav: torch.Tensor) -> torch.Tensor:
        """In place: songs whose peak |x| exceeds 1 are divided by it — the decode
        output guard of ``_decode_generate_music_pred_latents``
        (generate_music_decode.py:190-192).  wav fp32 [B, C, N] on the device."""
        assert wav.dtype == torch.float32 and wav.is_contiguous()
        B = wav.shape[0]
        peak = torch.empty(B, device=wav.device, dtype=torch.float32)
        check(lib().acehip_wav_peak_normalize(ptr(wav), B, wav.numel() // B, ptr(peak), stream_ptr()),
              "wav_peak_normalize")
        return wav

    @staticmethod
    def postprocess_(wav: torch.Tensor, normalization_db: Optional[float] = -1.0) -> torch.Tensor:
        """In place, one fused HIP pass pair per batch: the decode guard (divide a song by
        its peak when > 1, generate_music_decode.py:193-195) followed by the product's
        ``normalize_audio(audio, normalization_db)`` (audio_utils.py:24-62, applied at
        inference.py:674-679 when ``enable_normalization and normalization_db <= 0``);
        ``normalization_db=None`` = guard only.  Bit-identical to the two reference steps."""
        assert wav.dtype == torch.float32 and wav.is_contiguous()
        target = 0.0
        if normalization_db is not None:
            if normalization_db > 0.0:
                raise ValueError("normalization_db must be <= 0 (inference.py:674)")
            # torch promotes the python float to fp32 in target_amp / peak
            target = float(torch.tensor(10 ** (normalization_db / 20.0), dtype=torch.float32))
        B = wav.shape[0]
        peak = torch.empty(B, device=wav.device, dtype=torch.float32)
        check(lib().acehip_wav_postprocess(ptr(wav), B, wav.numel() // B, ptr(peak), 1, target, stream_ptr()),
              "wav_postprocess")
        return wav

    def decode(self, z: torch.Tensor):
        """diffusers-style: ``.decode(z).sample``."""
        return SimpleNamespace(sample=self.decode_tensor(z))

    def tiled_decode(self, latents: torch.Tensor, chunk_size: Optional[int] = None,
                     overlap: int = 64, offload_wav_to_cpu: Optional[bool] = None) -> torch.Tensor:
        """Handler ``tiled_decode`` contract (vae_decode.py:16-85): [B,64,T] →
        [B,2,T·hop].  The Oobleck decoder's receptive field (−8.2/+9.2 frames,
        SURVEY §8a a19) is inside the reference's 64-frame overlap, so its
        overlap-discard tiling equals an untiled decode; we decode untiled."""
        wav = self.decode_tensor(latents)
        # None = keep on the device here; the install() wrapper resolves None through the
        # handler's own policy first (_should_offload_wav_to_cpu, vae_decode.py:53-54)
        return wav.cpu() if offload_wav_to_cpu else wav

    def encode_tensor(self, wav: torch.Tensor, sample: bool = True,
                      generator: Optional[torch.Generator] = None,
                      eps: Optional[torch.Tensor] = None) -> torch.Tensor:
        """wav [B, 2, N] → latent [B, 64, N // hop] (mean + std·ε when sample); any
        N >= hop (AutoencoderOobleck's strided convs floor the length at every stage)."""
        if not self.with_encoder:
            raise RuntimeError("acehip: VAE created without encoder")
        wav = wav.to(device=self.device, dtype=torch.bfloat16).contiguous()
        B, _, N = wav.shape
        T = N // self.hop
        if eps is not None:
            eps = eps.to(device=self.device, dtype=torch.bfloat16).contiguous()
        elif sample:
            eps = torch.randn(B, self.cfg.decoder_input_channels, T, device=self.device,
                              dtype=torch.bfloat16, generator=generator)
        z = torch.empty(B, self.cfg.decoder_input_channels, T, device=self.device, dtype=torch.bfloat16)
        check(lib().acehip_vae_encode(self.h, ptr(wav), B, N, ptr(eps), ptr(z), stream_ptr()), "vae_encode")
        return z

    def tiled_encode(self, audio: torch.Tensor, chunk_size: Optional[int] = None,
                     overlap: Optional[int] = None, offload_latent_to_cpu: bool = True) -> torch.Tensor:
        """Handler ``tiled_encode`` contract (vae_encode.py:15-82, called by
        batch_prep.py:70 and conditioning_embed.py:58): audio [B, 2, N] or [2, N] →
        ``latent_dist.sample()`` latents [B, 64, N // hop] (or [64, N // hop]) in the
        VAE dtype, on the CPU when ``offload_latent_to_cpu`` (the reference default).

        ONE untiled encode of the whole batch instead of the reference's 30 s chunks
        with 2 s overlap (vae_encode_chunks.py:10-98, each chunk a separate encode and,
        by default, a device→host copy): the encoder's receptive field is inside the
        overlap, so the overlap-discard tiling computes the untiled mean
        (tests/test_gpu_long.py windows); ``chunk_size`` / ``overlap`` are accepted and
        ignored.  The Gaussian draw is one ``randn`` over the whole latent, where the
        reference draws per chunk — the same distribution, as in its own
        ``samples <= chunk_size`` branch.  Placement follows the reference: a source of at most
        ``chunk_size`` samples (default 30 s, 15 s on a GPU of ≤ 8 GB, vae_encode.py:46-53)
        comes back on the device whatever ``offload_latent_to_cpu`` says (vae_encode.py:62-68);
        longer ones are offloaded when it is set."""
        if chunk_size is None:
            # get_gpu_memory_gb (gpu_config.py:316-360): the MAX_CUDA_VRAM debug override first
            try:
                mem_gb = float(os.environ["MAX_CUDA_VRAM"])
            except (KeyError, ValueError):
                mem_gb = torch.cuda.get_device_properties(self.device).total_memory / 1024 ** 3
            chunk_size = 48000 * 15 if mem_gb <= 8 else 48000 * 30
        if overlap is None:
            overlap = 48000 * 2
        was_2d = audio.dim() == 2
        if was_2d:
            audio = audio.unsqueeze(0)
        if audio.dim() != 3 or audio.shape[1] != self.cfg.audio_channels:
            raise ValueError(f"acehip tiled_encode: expected [B, {self.cfg.audio_channels}, N] audio, "
                             f"got {tuple(audio.shape)}")
        if audio.shape[-1] > chunk_size and chunk_size - 2 * overlap <= 0:
            # the reference's chunked branch refuses a non-positive stride (vae_encode.py:70-72)
            raise ValueError(f"chunk_size {chunk_size} must be > 2 * overlap {overlap}")
        z = self.encode_tensor(audio, sample=True)
        if was_2d:
            z = z.squeeze(0)
        return z.cpu() if offload_latent_to_cpu and audio.shape[-1] > chunk_size else z

    def encode(self, wav: torch.Tensor):
        """diffusers-style: ``.encode(x).latent_dist.sample()`` / ``.mode()``."""
        be = self

        class _Dist:
            def sample(self, generator=None):
                return be.encode_tensor(wav, sample=True, generator=generator)

            def mode(self):
                return be.encode_tensor(wav, sample=False)
        return SimpleNamespace(latent_dist=_Dist())

    def close(self):
        if getattr(self, "h", None):
            lib().acehip_vae_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
