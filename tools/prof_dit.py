#!/usr/bin/env python3
"""Small full-size DiT driver for rocprofv3 passes (kernel trace / PMC):
builds the 24-layer runtime at the bench shape and runs a few forwards."""
import argparse, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip.config import DiTConfig, VAEConfig
from acehip.dit import DiTRuntime
from acehip.weights import synth_dit_weights, synth_vae_weights

p = argparse.ArgumentParser()
p.add_argument("--seconds", type=float, default=240)
p.add_argument("--forwards", type=int, default=2)
p.add_argument("--vae", action="store_true")
a = p.parse_args()
dev = torch.device("cuda:0")
cfg = DiTConfig()
T = int(a.seconds * 25); S = (T + 1) // 2
W = synth_dit_weights(cfg, seed=0, mode="bench", device=dev, dtype=torch.bfloat16, backend="torch")
rt = DiTRuntime(cfg, 0, max_S=S, max_Bc=2, max_Lenc=641)
rt.load(W); del W
g = torch.Generator(device=dev).manual_seed(0)
rt.set_condition(torch.randn(2, 641, 2048, device=dev, generator=g).bfloat16())
xt = torch.randn(1, T, 64, device=dev, generator=g).bfloat16()
ctx = torch.randn(1, T, 128, device=dev, generator=g).bfloat16()
t = torch.tensor([0.75], device=dev)
for _ in range(a.forwards):
    rt.forward(xt, ctx, t)
torch.cuda.synchronize()
if a.vae:
    from acehip.vae import OobleckBackend
    vc = VAEConfig()
    vae = OobleckBackend(vc, 0, max_T=T, with_encoder=False)
    vae.load(synth_vae_weights(vc, seed=0, mode="bench", with_encoder=False, device=dev,
                               dtype=torch.bfloat16, backend="torch"))
    vae.decode_tensor(torch.randn(1, 64, T, device=dev, generator=g).bfloat16())
    torch.cuda.synchronize()
print("done")
