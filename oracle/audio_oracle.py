"""CPU restatement of the decode output path — TEST ORACLE ONLY.

* ``decode_guard``: ``_decode_generate_music_pred_latents`` after the VAE
  (acestep/core/generation/handler/generate_music_decode.py:191-195): cast to
  fp32, per-song peak over (channels, samples), and when ANY song's peak > 1
  every song is divided by ``peak.clamp(min=1)``.
* ``normalize_audio``: acestep/audio_utils.py:24-62, applied per song at
  acestep/inference.py:674-679: peak of |x|; silence (< 1e-6) is returned
  unchanged; gain = 10^(db/20) / peak; x * gain.
"""
import torch


def decode_guard(wavs: torch.Tensor) -> torch.Tensor:
    if wavs.dtype != torch.float32:
        wavs = wavs.float()
    peak = wavs.abs().amax(dim=[1, 2], keepdim=True)
    if torch.any(peak > 1.0):
        wavs = wavs / peak.clamp(min=1.0)
    return wavs


def normalize_audio(audio: torch.Tensor, target_db: float = -1.0) -> torch.Tensor:
    a = audio.clone()
    peak = torch.max(torch.abs(a))
    if peak < 1e-6:
        return audio
    target_amp = 10 ** (target_db / 20.0)
    gain = target_amp / peak
    return a * gain
