#!/usr/bin/env python3
"""In-process A/B of the full-size Oobleck decode (240 s: T = 6000) between the
working-tree library and an alternative build (tools/ab_build.sh)."""
import ctypes, os, sys, statistics, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch
from acehip import _ffi
from acehip.config import VAEConfig
from acehip.vae import OobleckBackend
from acehip.weights import synth_vae_weights

dev = torch.device("cuda:0")
T = int(os.environ.get("VAE_T", "6000"))
cfg = VAEConfig()
W = synth_vae_weights(cfg, seed=0, mode="bench", with_encoder=False, device=dev, dtype=torch.bfloat16, backend="torch")
bes = {}
for name, path in [("tree", None)] + [(os.path.basename(p), p) for p in sys.argv[1:]]:
    if path is not None:
        lib = ctypes.CDLL(os.path.abspath(path))
        _ffi._declare(lib)
        _ffi._LIB = lib
    else:
        _ffi._LIB = None
        _ffi.lib()
    be = OobleckBackend(cfg, 0, max_T=T, with_encoder=False)
    be.load(W)
    bes[name] = (be, _ffi._LIB)
z = torch.randn(1, 64, T, device=dev).bfloat16()
outs, times = {}, {k: [] for k in bes}
for name, (be, lib) in bes.items():
    _ffi._LIB = lib
    outs[name] = be.decode_tensor(z).clone()
for _ in range(4):
    for name, (be, lib) in bes.items():
        _ffi._LIB = lib
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            be.decode_tensor(z)
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / 3)
print(json.dumps({k: {"ms": round(statistics.median(v), 2),
                      "maxdiff_vs_tree": float((outs[k] - outs["tree"]).abs().max())} for k, v in times.items()}))
