#!/usr/bin/env python3
"""Measure the HIP VAE against the two oracle precisions (sets the bars in tests/test_vae.py and
tests/test_gpu_long.py): the fp32 restatement (oracle/vae_oracle.decode) and the bf16-storage
restatement run as torch on the GPU (decode_bf16_storage: bf16 activations between ops, fp32
math inside each, as the reference's bf16 VAE stores them).  Prints one JSON line per case."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

from conftest import rel_l2  # noqa: E402
from acehip.config import VAEConfig  # noqa: E402
from acehip.vae import OobleckBackend  # noqa: E402
from acehip.weights import synth_vae_weights  # noqa: E402
from oracle import vae_oracle  # noqa: E402

dev = torch.device("cuda:0")
CORE, CTX = 32, 40


def main():
    for name, cfg, T in (("tiny", VAEConfig.tiny(), 7), ("full", VAEConfig(), 8), ("full", VAEConfig(), 6000)):
        W = synth_vae_weights(cfg, seed=5, mode="parity", with_encoder=True)
        Wd = {k: v.to(dev) for k, v in W.items()}
        be = OobleckBackend(cfg, 0, max_T=max(T, 16), with_encoder=True)
        be.load(Wd)
        g = torch.Generator(device=dev).manual_seed(T + 1)
        z = torch.randn(1, 64, T, device=dev, generator=g).bfloat16()
        wins = [(0, T)] if T < 100 else [(max(0, c0 - CTX), min(T, c0 + CORE + CTX)) for c0 in (0, T // 2 - 16, T - 32)]
        for lo, hi in wins:
            zw = z[:, :, lo:hi].contiguous()
            out = be.decode_tensor(zw).float()
            with torch.no_grad():
                r32 = vae_oracle.decode(Wd, cfg, zw.float())
                rb = vae_oracle.decode_bf16_storage(Wd, cfg, zw)
                rn = vae_oracle.decode({k: v.bfloat16() for k, v in Wd.items()}, cfg, zw).float()
            torch.cuda.synchronize()
            print(json.dumps({"case": f"decode {name} T={T} win=[{lo},{hi})",
                              "hip_vs_fp32": rel_l2(out.cpu(), r32.cpu()), "hip_vs_bf16_storage": rel_l2(out.cpu(), rb.cpu()),
                              "bf16_storage_vs_fp32": rel_l2(rb.cpu(), r32.cpu()),
                              "naive_bf16_vs_fp32": rel_l2(rn.cpu(), r32.cpu())}), flush=True)
        if T < 100:
            wav = (0.3 * torch.randn(2, 2, 3 * 1920 + 777, device=dev, generator=g)).bfloat16()
            m = be.encode_tensor(wav, sample=False).float()
            with torch.no_grad():
                m32 = vae_oracle.encode_sample(Wd, cfg, wav.float())
                mb = vae_oracle.encode_mean_bf16_storage(Wd, cfg, wav)
            print(json.dumps({"case": f"encode {name}", "hip_vs_fp32": rel_l2(m.cpu(), m32.cpu()),
                              "hip_vs_bf16_storage": rel_l2(m.cpu(), mb.cpu()),
                              "bf16_storage_vs_fp32": rel_l2(mb.cpu(), m32.cpu())}), flush=True)
        be.close()


if __name__ == "__main__":
    main()
