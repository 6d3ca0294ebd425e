#!/usr/bin/env python3
"""DiT part of a 240 s song (27 CFG steps through AceStepDiTBackend.generate_audio) timed
under several environment settings, interleaved in ONE process.

usage: ab_env_song.py 'NAME=VAL[,NAME=VAL]' ['...' ...]   (first = baseline)
SONG_SECONDS (default 240) and SONG_TURBO=1 (8 turbo steps, Bc = 1, no CFG) pick the song."""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip._ffi import reload_knobs  # noqa: E402  (the library reads its switches once)
from acehip.config import DiTConfig  # noqa: E402
from acehip.dit import AceStepDiTBackend, DiTRuntime  # noqa: E402
from acehip.weights import synth_dit_weights  # noqa: E402

settings = [dict(kv.split("=") for kv in a.split(",") if kv) for a in sys.argv[1:]] or [{}]
dev = torch.device("cuda:0")
cfg = DiTConfig()
T = int(float(os.environ.get("SONG_SECONDS", "240")) * 25)
S = (T + 1) // 2
TURBO = os.environ.get("SONG_TURBO", "0") == "1"
W = synth_dit_weights(cfg, seed=0, mode="bench", device=dev, dtype=torch.bfloat16, backend="torch")
rt = DiTRuntime(cfg, 0, max_S=S, max_Bc=2, max_Lenc=641)
rt.load(W)
del W
g = torch.Generator(device=dev).manual_seed(0)
null = torch.randn(1, 1, cfg.hidden_size, device=dev, generator=g).bfloat16()
be = AceStepDiTBackend(rt, null, is_turbo=TURBO)
enc = torch.randn(1, 641, cfg.hidden_size, device=dev, generator=g).bfloat16()
ctx = torch.randn(1, T, 128, device=dev, generator=g).bfloat16()


def song():
    if TURBO:
        return be.generate_audio(encoder_hidden_states=enc, context_latents=ctx, infer_steps=8, shift=3.0,
                                 seed=1)["target_latents"]
    return be.generate_audio(encoder_hidden_states=enc, context_latents=ctx, infer_steps=27,
                             diffusion_guidance_sale=7.0, shift=3.0, seed=1)["target_latents"]


outs, times = [], [[] for _ in settings]
for st in settings:
    os.environ.update(st)
    reload_knobs()
    outs.append(song().float().clone())
    for k in st:
        os.environ.pop(k)
        reload_knobs()
for _ in range(int(os.environ.get("ROUNDS", "3"))):
    for i, st in enumerate(settings):
        os.environ.update(st)
        reload_knobs()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        song()
        torch.cuda.synchronize()
        times[i].append((time.perf_counter() - t0) * 1e3)
        for k in st:
            os.environ.pop(k)
            reload_knobs()
for i, st in enumerate(settings):
    same = torch.equal(outs[i], outs[0])
    print(f"{','.join(f'{a}={b}' for a, b in st.items()) or 'default'}: DiT song {statistics.median(times[i]):.1f} ms "
          f"(min {min(times[i]):.1f}; bit-identical to baseline: {same})", flush=True)
