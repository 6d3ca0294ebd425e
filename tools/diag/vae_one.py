#!/usr/bin/env python3
"""One full-size (240 s, T = 6000) Oobleck decode, for rocprofv3 counter passes."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip.config import VAEConfig  # noqa: E402
from acehip.vae import OobleckBackend  # noqa: E402
from acehip.weights import synth_vae_weights  # noqa: E402

T = int(os.environ.get("VAE_T", "6000"))
dev = torch.device("cuda:0")
cfg = VAEConfig()
vae = OobleckBackend(cfg, 0, max_T=T, with_encoder=False)
vae.load(synth_vae_weights(cfg, seed=0, mode="bench", with_encoder=False, device=dev, dtype=torch.bfloat16,
                           backend="torch"))
z = torch.randn(1, 64, T, device=dev).bfloat16()
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1):
    vae.decode_tensor(z)
torch.cuda.synchronize()
print("ok")
