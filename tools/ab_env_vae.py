#!/usr/bin/env python3
"""240 s VAE decode timed under several environment settings, interleaved in ONE process
(the library reads its A/B knobs per launch).

usage: ab_env_vae.py 'NAME=VAL[,NAME=VAL]' ['...' ...]   (first = baseline)"""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip._ffi import reload_knobs  # noqa: E402  (the library reads its switches once)
from acehip.config import VAEConfig  # noqa: E402
from acehip.vae import OobleckBackend  # noqa: E402
from acehip.weights import synth_vae_weights  # noqa: E402

settings = [dict(kv.split("=") for kv in a.split(",") if kv) for a in sys.argv[1:]] or [{}]
dev = torch.device("cuda:0")
T = int(os.environ.get("VAE_T", "6000"))
vc = VAEConfig()
vae = OobleckBackend(vc, 0, max_T=T, with_encoder=False)
vae.load(synth_vae_weights(vc, seed=0, mode="bench", with_encoder=False, device=dev, dtype=torch.bfloat16,
                           backend="torch"))
g = torch.Generator(device=dev).manual_seed(0)
z = torch.randn(1, 64, T, device=dev, generator=g).bfloat16()
outs, times = [], [[] for _ in settings]
for st in settings:
    os.environ.update(st)
    reload_knobs()
    outs.append(vae.decode_tensor(z).float().clone())
    for k in st:
        os.environ.pop(k)
        reload_knobs()
for _ in range(5):
    for i, st in enumerate(settings):
        os.environ.update(st)
        reload_knobs()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        vae.decode_tensor(z)
        torch.cuda.synchronize()
        times[i].append((time.perf_counter() - t0) * 1e3)
        for k in st:
            os.environ.pop(k)
            reload_knobs()
for i, st in enumerate(settings):
    print(f"{','.join(f'{a}={b}' for a, b in st.items()) or 'default'}: decode {statistics.median(times[i]):.2f} ms "
          f"(min {min(times[i]):.2f}; bit-identical to baseline: {torch.equal(outs[i], outs[0])})", flush=True)
