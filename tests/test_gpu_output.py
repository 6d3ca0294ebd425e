"""The output leg after the decode on the GPU: the fused guard + normalize +
PCM16 pack (acehip_wav_postprocess_pcm16) against the reference's own steps, the asynchronous
WAV writer, and the bf16 rounding of decode(z).sample."""
import wave

import numpy as np
import pytest
import torch

from acehip.config import VAEConfig
from acehip.weights import synth_vae_weights

pytestmark = pytest.mark.gpu


def _ref_leg(wav_cpu, db=-1.0):
    """generate_music_decode.py:188-195 (guard, per song) then audio_utils.normalize_audio
    (inference.py:674-679) per song, then the soundfile PCM16 conversion of [samples, channels]
    frames: rint(clamp(x, -1, 1) * 32767)."""
    w = wav_cpu.float()
    peak = w.abs().amax(dim=[1, 2], keepdim=True)
    if torch.any(peak > 1.0):
        w = w / peak.clamp(min=1.0)
    out, frames = [], []
    for b in range(w.shape[0]):
        a = w[b]
        pk = torch.max(torch.abs(a))
        if not pk < 1e-6:
            a = a.clone() * (10 ** (db / 20.0) / pk)
        out.append(a)
        frames.append(torch.round(torch.clamp(a.t(), -1.0, 1.0) * 32767.0).to(torch.int16))
    return torch.stack(out), torch.stack(frames)


@pytest.mark.parametrize("C,N", [(2, 4096), (2, 11_520_000), (1, 1000)])
def test_postprocess_pcm16_bit_exact(gpu_device, C, N):
    from acehip.output import postprocess_pcm16_
    g = torch.Generator().manual_seed(N + C)
    wav = torch.randn(3, C, N, generator=g) * 0.3
    wav[0] *= 5.0                                  # peak > 1: the guard divides first
    wav[2] *= 1e-8                                 # silence: normalize_audio returns it unchanged
    ref_w, ref_pcm = _ref_leg(wav)
    d = wav.to(gpu_device).contiguous()
    pcm = postprocess_pcm16_(d, -1.0)
    torch.cuda.synchronize()
    assert pcm.shape == (3, N, C) and pcm.dtype == torch.int16
    assert torch.equal(d.cpu(), ref_w)             # the fp32 tensor the reference returns, bit-exact
    assert torch.equal(pcm.cpu(), ref_pcm)         # the PCM16 frames soundfile would encode
    # same fp32 result as the unfused postprocess pass pair (acehip_wav_postprocess)
    from acehip import _ffi as ff
    from acehip.output import target_amp
    d2 = wav.to(gpu_device).contiguous()
    peak = torch.empty(3, device=gpu_device)
    ff.check(ff.lib().acehip_wav_postprocess(ff.ptr(d2), 3, C * N, ff.ptr(peak), 1, target_amp(-1.0),
                                             ff.stream_ptr()), "wav_postprocess")
    torch.cuda.synchronize()
    assert torch.equal(d2.cpu(), ref_w)


def test_pcm16_clamp_and_guard_only(gpu_device):
    """normalization off (None): the guard alone, and samples outside [-1, 1] cannot occur after
    it; the clamp is exercised on a song whose peak is exactly 1 (no division)."""
    from acehip.output import postprocess_pcm16_
    x = torch.tensor([[[1.0, -1.0, 0.49999, -0.25, 0.0, 1.0 / 65534, -1.0 / 65534, 0.999]]]).repeat(1, 2, 1)
    d = x.to(gpu_device).contiguous()
    pcm = postprocess_pcm16_(d, None)
    torch.cuda.synchronize()
    exp = torch.round(torch.clamp(x[0].t(), -1, 1) * 32767).to(torch.int16)
    assert torch.equal(pcm[0].cpu(), exp)
    assert torch.equal(d.cpu(), x)


def test_audio_writer_files(gpu_device, tmp_path):
    from acehip.output import AudioWriter
    N = 48000
    writer = AudioWriter(gpu_device, N, channels=2, slots=2)
    g = torch.Generator().manual_seed(3)
    songs = [torch.randn(2, 2, N, generator=g) * s for s in (0.2, 2.0)]
    paths = []
    for i, w in enumerate(songs):
        d = w.to(gpu_device).contiguous()
        ps = [str(tmp_path / f"s{i}_{b}.wav") for b in range(2)]
        writer.submit(d, ps)
        paths += ps
    written = writer.flush()
    writer.close()
    assert sorted(written) == sorted(paths)
    k = 0
    for w in songs:
        _, ref = _ref_leg(w)
        for b in range(2):
            with wave.open(paths[k], "rb") as f:
                assert f.getnchannels() == 2 and f.getsampwidth() == 2 and f.getframerate() == 48000
                assert f.getnframes() == N
                got = np.frombuffer(f.readframes(N), dtype="<i2").reshape(N, 2)
            assert np.array_equal(got, ref[b].numpy())
            k += 1


def test_decode_sample_is_bf16_rounded(gpu_device):
    """decode(z).sample holds bf16 values, as the reference's bf16 VAE output upcast by the
    handler (init_service_loader.py:132-134, generate_music_decode.py:188-189)."""
    from acehip.vae import OobleckBackend
    cfg = VAEConfig.tiny()
    W = synth_vae_weights(cfg, seed=2, mode="parity", with_encoder=False)
    be = OobleckBackend(cfg, gpu_device.index or 0, max_T=16, with_encoder=False)
    be.load({k: v.to(gpu_device) for k, v in W.items()})
    z = torch.randn(1, 64, 16, generator=torch.Generator().manual_seed(1)).bfloat16().to(gpu_device)
    wav = be.decode(z).sample
    torch.cuda.synchronize()
    assert wav.dtype == torch.float32
    assert torch.equal(wav, wav.bfloat16().float())
    assert wav.abs().max() > 0
    be.close()
