#!/usr/bin/env python3
"""Where a ru8_kernel tile's time goes (the C = 128 residual unit, snake-in variant, of the 240 s
decode): runs the full-size decode on an RU8_STAMPS build (tools/ab_build.sh WT ru8stamps
-DRU8_STAMPS) and reads the stamps of the LAST ru8 launch of the decode (block 4, unit 2:
11.52 M rows, dilation 9), one steady-state tile (each block's second) per block.

Per K-tile kt, medians over blocks, in shader-clock cycles:
  mfma_wait   MFMA wave 0 at barrier kt (arrival → release)
  mfma_work   MFMA wave 0 from barrier kt's release to barrier kt+1's arrival (its K-tile work)
  w_vmwait    the W helper's counted vmcnt wait before barrier kt (W(kt) and its window landing)
  w_late      W helper's arrival at barrier kt − MFMA wave 0's arrival (> 0: the MFMA waves wait for W)
  win_late    window helper 0's arrival − MFMA wave 0's arrival
plus the epilogue-2 cycles, the tile's cycles and the effective shader clock (cycles ÷ real time).

usage: ru8_stamps.py [tools/ab/libacehip_ru8stamps.so]"""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from acehip import _ffi  # noqa: E402
from acehip.config import VAEConfig  # noqa: E402
from acehip.vae import OobleckBackend  # noqa: E402
from acehip.weights import synth_vae_weights  # noqa: E402

RST_BLK, SLOTS = 1024, 36
LIB = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "tools", "ab", "libacehip_ru8stamps.so")


def main():
    lib = ctypes.CDLL(os.path.abspath(LIB))
    _ffi._declare(lib)
    _ffi._LIB = lib
    lib.acehip_diag_ru8_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    T = int(os.environ.get("VAE_T", "6000"))
    cfg = VAEConfig()
    W = synth_vae_weights(cfg, seed=0, mode="bench", with_encoder=False, device=dev, dtype=torch.bfloat16,
                          backend="torch")
    be = OobleckBackend(cfg, 0, max_T=T, with_encoder=False)
    be.load(W)
    z = torch.randn(1, 64, T, device=dev).bfloat16()
    be.decode_tensor(z)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    lib.acehip_diag_ru8_stamps_clear()
    e0.record()
    be.decode_tensor(z)
    e1.record()
    torch.cuda.synchronize()
    buf = np.zeros(RST_BLK * 3 * SLOTS, dtype=np.uint64)
    assert lib.acehip_diag_ru8_stamps(buf.ctypes.data) == 0
    st = buf.reshape(RST_BLK, 3, SLOTS).astype(np.int64)
    rows = []
    for b in range(RST_BLK):
        m, w, h = st[b, 0], st[b, 1], st[b, 2]
        if m[0] == 0 or w[0] == 0 or np.any(np.diff(m[:34]) < 0) or np.any(np.diff(w[:32]) < 0):
            continue
        rows.append((m, w, h))
    out = {"decode_ms": round(e0.elapsed_time(e1), 2), "blocks": len(rows), "per_kt": []}
    med = lambda xs: int(statistics.median(xs))  # noqa: E731
    for kt in range(16):
        nxt = 32 if kt == 15 else 2 * kt + 2
        r = {"kt": kt,
             "mfma_wait": med([m[2 * kt + 1] - m[2 * kt] for m, _, _ in rows]),
             "mfma_work": med([m[nxt] - m[2 * kt + 1] for m, _, _ in rows]),
             "w_vmwait": med([w[2 * kt + 1] - w[2 * kt] for _, w, _ in rows]),
             "w_late": med([w[2 * kt + 1] - m[2 * kt] for m, w, _ in rows])}
        hv = [h[2 * kt + 1] - m[2 * kt] for m, _, h in rows if h[0] != 0]
        r["win_late"] = med(hv) if hv else None
        out["per_kt"].append(r)
    tile = [m[33] - m[1] for m, _, _ in rows]
    real = [(m[35] - m[34]) / 100e6 for m, _, _ in rows]       # s_memrealtime: 100 MHz
    out["epilogue2"] = med([m[33] - m[32] for m, _, _ in rows])
    out["tile_cycles"] = med(tile)
    out["tile_us"] = round(statistics.median(real) * 1e6, 2)
    out["clock_GHz"] = round(statistics.median([c / r / 1e9 for c, r in zip(tile, real) if r > 0]), 3)
    out["mfma_cycles_ideal_per_kt"] = 4 * 8 * 2 * 16     # 64 MFMAs 16x16x32 per wave per K-tile
    s = sum(r["mfma_wait"] for r in out["per_kt"])
    out["sum_mfma_wait"] = s
    out["sum_mfma_work"] = sum(r["mfma_work"] for r in out["per_kt"])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
