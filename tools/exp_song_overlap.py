#!/usr/bin/env python3
"""Songs back to back on one GPU: sequential (DiT k, decode k, DiT k+1, …) against the decode of
song k on a second stream while song k+1's DiT runs on the first (the VAE's LDS-heavy persistent
grids filling the DiT kernels' partial last rounds).  240 s songs, 27 CFG steps, synthetic
conditioning (encoder states given directly).  Prints s/song for both, interleaved rounds.

usage: exp_song_overlap.py [songs per round (4)] [rounds (2)]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402

from acehip.config import DiTConfig, VAEConfig  # noqa: E402
from acehip.dit import AceStepDiTBackend, DiTRuntime  # noqa: E402
from acehip.vae import OobleckBackend  # noqa: E402
from acehip.weights import synth_dit_weights, synth_null_condition, synth_vae_weights  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
R = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dev = torch.device("cuda:0")
cfg, vcfg = DiTConfig(), VAEConfig()
T = 6000
S = T // 2
rt = DiTRuntime(cfg, 0, max_S=S, max_Bc=2, max_Lenc=641)
rt.load(synth_dit_weights(cfg, seed=0, mode="bench", device=dev, dtype=torch.bfloat16, backend="torch"))
be = AceStepDiTBackend(rt, synth_null_condition(cfg, seed=0, device=dev, dtype=torch.bfloat16, backend="torch"))
vae = OobleckBackend(vcfg, 0, max_T=T)
vae.load(synth_vae_weights(vcfg, seed=0, mode="bench", device=dev, dtype=torch.bfloat16, backend="torch"))
g = torch.Generator(device=dev).manual_seed(0)
enc = torch.randn(1, 641, cfg.hidden_size, device=dev, generator=g).bfloat16()
ctx = torch.cat([torch.randn(1, T, 64, device=dev, generator=g), torch.ones(1, T, 64, device=dev)], -1).bfloat16()
kw = dict(encoder_hidden_states=enc, context_latents=ctx.contiguous(), infer_steps=27, diffusion_guidance_sale=7.0,
          shift=3.0, infer_method="ode")
side = torch.cuda.Stream(device=dev)
wav_out = [None, None]


def dit(i):
    return be.generate_audio(seed=i, **kw)["target_latents"]


def sequential(n):
    for i in range(n):
        lat = dit(i)
        w = vae.decode_tensor(lat.transpose(1, 2))
        vae.postprocess_(w, -1.0)
        wav_out[i & 1] = w


def overlapped(n):
    main = torch.cuda.current_stream(dev)
    prev = None
    for i in range(n + 1):
        if prev is not None:                       # decode song i-1 on the side stream
            lat_p, ev = prev
            side.wait_event(ev)
            with torch.cuda.stream(side):
                w = vae.decode_tensor(lat_p.transpose(1, 2))
                vae.postprocess_(w, -1.0)
                wav_out[i & 1] = w
            lat_p.record_stream(side)
        if i < n:
            lat = dit(i)
            ev = main.record_event()
            prev = (lat, ev)
    main.wait_stream(side)


for fn in (sequential, overlapped):
    fn(1)
torch.cuda.synchronize()
res = {"sequential": [], "overlapped": []}
for _ in range(R):
    for name, fn in (("sequential", sequential), ("overlapped", overlapped)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(N)
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / N)
        print(f"{name}: {res[name][-1] * 1e3:.1f} ms/song", flush=True)
print({k: round(min(v) * 1e3, 1) for k, v in res.items()})
