#!/usr/bin/env python3
"""Record the reference's own VAE-seam arithmetic that runs without diffusers (this container only;
the reference never travels):

1. The tiled decode (``acestep/core/generation/handler/vae_decode_chunks.py:13-166``, loaded with a
   ``loguru`` stub): ``_tiled_decode_inner`` → ``_tiled_decode_gpu`` / ``_tiled_decode_offload_cpu``
   driven with a stand-in VAE (hop 1920) that records every window it is asked to decode and
   returns audio tagged with (window number, sample index within the window) (latent frame t
   carries the value t, so the stand-in knows where its window starts).  Stored per (T, chunk,
   overlap, path): the windows [win_start, win_end), the range of each window's samples the
   reference kept (read off its stitched output), and whether that output is exactly the samples
   0 … 1920·T − 1 in order (tiled ≡ untiled for any decoder whose receptive field is inside the
   overlap).  ``tests/test_gpu_long.py`` replays the recorded windows through
   the HIP decoder and stitches them with the recorded trims.
2. The weight-norm fusion of the reference's VAE converter (``acestep/models/mlx/vae_convert.py:19-34``,
   ``_fuse_weight_norm``, numpy) on seeded Conv1d / ConvTranspose1d ``weight_g`` / ``weight_v``
   tensors: inputs and fused outputs, against which ``tests/test_vae.py`` checks the oracle's
   ``fuse_weight_norm``.

3. The decode output guard (``generate_music_decode.py:98-201``
   ``_decode_generate_music_pred_latents``, ``acestep.gpu_config`` stubbed) with a stand-in bf16 VAE:
   the waveform it returns and the guarded fp32 ``pred_wavs`` the reference hands on.

4. ``normalize_audio`` (``acestep/audio_utils.py:24-62``, torchaudio stubbed) on seeded songs.

Writes ``tests/golden/vae_seam.json``, ``vae_weight_norm.safetensors``, ``decode_guard.safetensors``
and ``normalize_audio.safetensors``."""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch
from safetensors.torch import save_file

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "tests", "golden")
REF = "/root/reference/acestep"
HOP = 1920


def _load(path, name):
    if "loguru" not in sys.modules:
        m = types.ModuleType("loguru")

        class _L:
            def __getattr__(self, _):
                return lambda *a, **k: None
        m.logger = _L()
        sys.modules["loguru"] = m
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


TAG = float(2 ** 32)


class IndexVae:
    """decode(z).sample for z [1, 64, L] whose channel 0 holds the global frame index: audio
    [1, 2, L·1920] whose samples are (call number)·2³² + (sample index within the window)
    (float64, exact), so the stitched output tells which window and which of its samples the
    reference kept at every position."""

    def __init__(self):
        self.calls = []

    def decode(self, z):
        w0, L = int(z[0, 0, 0].item()), z.shape[-1]
        n = len(self.calls)
        self.calls.append((w0, w0 + L))
        a = n * TAG + torch.arange(L * HOP, dtype=torch.float64)
        return types.SimpleNamespace(sample=a.view(1, 1, -1).repeat(1, 2, 1))


def record_tiling():
    mod = _load(os.path.join(REF, "core/generation/handler/vae_decode_chunks.py"), "_ref_vae_decode_chunks")

    class Host(mod.VaeDecodeChunksMixin):
        def __init__(self):
            self.vae = IndexVae()
            self.disable_tqdm = True

        def _empty_cache(self):
            pass

    out = []
    for T in (250, 641, 1000, 6000, 15000):
        for chunk in (512, 384, 256, 128):
            for offload in (False, True):
                h = Host()
                z = torch.zeros(1, 64, T, dtype=torch.float64)
                z[0, 0] = torch.arange(T, dtype=torch.float64)
                wav = h._tiled_decode_inner(z, chunk, 64, offload)[0, 0]
                wid = torch.floor(wav / TAG)
                local = wav - wid * TAG
                starts = torch.tensor([c[0] * HOP for c in h.vae.calls], dtype=torch.float64)
                glob = starts[wid.long()] + local
                exact = wav.numel() == T * HOP and bool(torch.equal(glob, torch.arange(T * HOP, dtype=torch.float64)))
                # the samples the reference kept of each window: [first, last + 1) of its own indices
                keep = []
                for n in range(len(h.vae.calls)):
                    sel = local[wid == n]
                    keep.append([int(sel.min().item()), int(sel.max().item()) + 1] if sel.numel() else [0, 0])
                    assert sel.numel() == keep[-1][1] - keep[-1][0], "kept samples of a window are contiguous"
                out.append({"T": T, "chunk": chunk, "overlap": 64, "offload_wav_to_cpu": offload,
                            "windows": [list(c) for c in h.vae.calls], "keep": keep,
                            "stitched_is_untiled": exact, "decoded_frames": sum(e - s for s, e in h.vae.calls)})
    return out


class IndexEncVae:
    """encode(x).latent_dist.sample() for audio [1, 2, N] whose channel 0 holds the global sample
    index: latents [1, 64, N // 1920] tagged (call number)·2³² + (frame index within the window)."""

    def __init__(self):
        self.calls = []
        self.dtype = torch.float64

    def encode(self, x):
        s0, N = int(x[0, 0, 0].item()), x.shape[-1]
        n = len(self.calls)
        self.calls.append((s0, s0 + N))
        lat = n * TAG + torch.arange(N // HOP, dtype=torch.float64)
        return types.SimpleNamespace(latent_dist=types.SimpleNamespace(
            sample=lambda: lat.view(1, 1, -1).repeat(1, 64, 1)))


def record_encode_tiling():
    """vae_encode_chunks.py:10-98 (chunks of 30 s / 15 s, overlap 2 s, both paths)."""
    mod = _load(os.path.join(REF, "core/generation/handler/vae_encode_chunks.py"), "_ref_vae_encode_chunks")

    class Host(mod.VaeEncodeChunksMixin):
        def __init__(self):
            self.vae = IndexEncVae()
            self.disable_tqdm = True
            self.device = "cpu"

    out = []
    for T in (1500, 6000, 15000):
        N = T * HOP
        for chunk in (48000 * 30, 48000 * 15):
            overlap = 48000 * 2
            for offload in (False, True):
                h = Host()
                x = torch.zeros(1, 2, N, dtype=torch.float64)
                x[0, 0] = torch.arange(N, dtype=torch.float64)
                stride = chunk - 2 * overlap
                steps = -(-N // stride)
                fn = h._tiled_encode_offload_cpu if offload else h._tiled_encode_gpu
                lat = fn(x, 1, N, stride, overlap, steps, chunk)[0, 0]
                wid = torch.floor(lat / TAG)
                local = lat - wid * TAG
                starts = torch.tensor([c[0] // HOP for c in h.vae.calls], dtype=torch.float64)
                exact = lat.numel() == T and bool(torch.equal(starts[wid.long()] + local,
                                                              torch.arange(T, dtype=torch.float64)))
                keep = []
                for n in range(len(h.vae.calls)):
                    sel = local[wid == n]
                    keep.append([int(sel.min().item()), int(sel.max().item()) + 1] if sel.numel() else [0, 0])
                out.append({"T": T, "chunk": chunk, "overlap": overlap, "offload_latent_to_cpu": offload,
                            "windows": [list(c) for c in h.vae.calls], "keep": keep, "stitched_is_untiled": exact})
    return out


def record_decode_guard():
    """generate_music_decode.py:98-201 `_decode_generate_music_pred_latents` (loguru and
    acestep.gpu_config stubbed) with a stand-in bf16 VAE returning a fixed waveform per song:
    the input waveform and the guarded fp32 `pred_wavs` the reference hands on."""
    if "acestep.gpu_config" not in sys.modules:
        for name in ("acestep", "acestep.gpu_config"):
            sys.modules.setdefault(name, types.ModuleType(name))
        sys.modules["acestep.gpu_config"].get_effective_free_vram_gb = lambda: 100.0
    mod = _load(os.path.join(REF, "core/generation/handler/generate_music_decode.py"), "_ref_generate_music_decode")
    g = torch.Generator().manual_seed(11)
    T = 4
    wav = torch.randn(4, 2, T * HOP, generator=g)
    wav[0] *= 2.5                                   # peak > 1: divided by its peak
    wav[1] *= 0.2                                   # below 1: untouched
    wav[2] *= 1e-6                                  # near silence
    wav[3] = wav[3] / wav[3].abs().max()            # exactly 1 after the bf16 cast? (kept as is)
    wav = wav.bfloat16()

    class StandInVae:
        dtype = torch.bfloat16

        def decode(self, z):
            assert z.dtype == torch.bfloat16 and z.shape == (4, 64, T)
            return types.SimpleNamespace(sample=wav.clone())

        def parameters(self):
            return iter([torch.zeros(1)])

    import contextlib

    class Host(mod.GenerateMusicDecodeMixin):
        def __init__(self):
            self.vae = StandInVae()
            self.device = "cpu"
            self.use_mlx_vae = False
            self.mlx_vae = None
            self.current_offload_cost = 0.0

        @contextlib.contextmanager
        def _load_model_context(self, name):
            yield

        def _empty_cache(self):
            pass

        def _memory_allocated(self):
            return 0

        def _max_memory_allocated(self):
            return 0

    lat = torch.randn(4, T, 64, generator=g).bfloat16()
    out, lat_cpu, _ = Host()._decode_generate_music_pred_latents(lat, None, False, {"total_time_cost": 0.0})
    assert out.dtype == torch.float32
    return {"wav_bf16": wav, "pred_wavs": out.contiguous()}


def record_normalize_audio():
    """acestep/audio_utils.py:24-62 `normalize_audio` (torchaudio stubbed: only AudioSaver uses it)
    on seeded songs of several loudness levels and target dB: inputs and outputs."""
    sys.modules.setdefault("torchaudio", types.ModuleType("torchaudio"))
    mod = _load(os.path.join(REF, "audio_utils.py"), "_ref_audio_utils")
    g = torch.Generator().manual_seed(5)
    t = {}
    for i, (scale, db) in enumerate([(3.0, -1.0), (0.3, -1.0), (1e-8, -1.0), (0.7, -6.0), (0.05, 0.0)]):
        a = torch.randn(2, 4800, generator=g) * scale
        t[f"case{i}.in"] = a
        t[f"case{i}.db"] = torch.tensor([db])
        t[f"case{i}.out"] = mod.normalize_audio(a, db).clone()   # silence comes back as the input object
    return t


def record_weight_norm():
    mod = _load(os.path.join(REF, "models/mlx/vae_convert.py"), "_ref_vae_convert")
    rng = np.random.Generator(np.random.PCG64(7))
    t = {}
    # Conv1d [out, in, k] (g [out, 1, 1]) and ConvTranspose1d [in, out, 2s] (g [in, 1, 1]) shapes of
    # the Oobleck decoder: conv1 k7, a residual k7 / k1, a ConvTranspose stride 2 / 10, conv2 k7
    shapes = {"conv1": (32, 16, 7), "res_k7": (32, 32, 7), "res_k1": (32, 32, 1), "convt_s2": (32, 16, 4),
              "convt_s10": (32, 16, 20), "conv2": (2, 32, 7)}
    for name, shp in shapes.items():
        v = rng.standard_normal(shp).astype(np.float32) * 0.02
        g = (np.linalg.norm(v.reshape(shp[0], -1), axis=1) * rng.uniform(0.5, 1.5, shp[0])).astype(np.float32)
        g = g.reshape(shp[0], 1, 1)
        w = mod._fuse_weight_norm(g, v)
        t[f"{name}.weight_g"] = torch.from_numpy(np.ascontiguousarray(g))
        t[f"{name}.weight_v"] = torch.from_numpy(np.ascontiguousarray(v))
        t[f"{name}.fused"] = torch.from_numpy(np.ascontiguousarray(w.astype(np.float32)))
    return t


def main():
    os.makedirs(OUT, exist_ok=True)
    tiling = record_tiling()
    enc = record_encode_tiling()
    with open(os.path.join(OUT, "vae_seam.json"), "w") as f:
        json.dump({"reference": "acestep/core/generation/handler/vae_decode_chunks.py:13-166",
                   "generator": "tools/record_vae_seam.py", "hop": HOP, "cases": tiling,
                   "encode_reference": "acestep/core/generation/handler/vae_encode_chunks.py:10-98",
                   "encode_cases": enc}, f)
    print("encode cases", len(enc), "not exact", sum(not c["stitched_is_untiled"] for c in enc))
    save_file(record_weight_norm(), os.path.join(OUT, "vae_weight_norm.safetensors"),
              metadata={"reference": "acestep/models/mlx/vae_convert.py:19-34 (_fuse_weight_norm)",
                        "generator": "tools/record_vae_seam.py"})
    save_file(record_decode_guard(), os.path.join(OUT, "decode_guard.safetensors"),
              metadata={"reference": "acestep/core/generation/handler/generate_music_decode.py:98-201",
                        "generator": "tools/record_vae_seam.py"})
    save_file(record_normalize_audio(), os.path.join(OUT, "normalize_audio.safetensors"),
              metadata={"reference": "acestep/audio_utils.py:24-62 (normalize_audio)",
                        "generator": "tools/record_vae_seam.py"})
    bad = [c for c in tiling if not c["stitched_is_untiled"]]
    print(f"wrote {len(tiling)} tiling cases ({len(bad)} not exact) and the weight-norm fixture")


if __name__ == "__main__":
    main()
