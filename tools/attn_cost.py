#!/usr/bin/env python3
"""Cost model of the 64-row-per-wave attention kernel: time vs KV tiles per unit and vs
units per CU, so the per-unit fixed cost (Q load, first-tile latency, epilogue) and the
per-tile cost can be separated.  Runs attn_pw_kernel on the cross-attention path
(window < 0, Sk != Sq) with Sk = 64·n keys, and the band layer at B = 1..4.

usage: attn_cost.py            (prints one JSON line per point)
"""
import json
import math
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip import _ffi as ff  # noqa: E402

dev = torch.device("cuda:0")
f = ff.lib().acehip_attention_bf16
os.environ["ACEHIP_ATTN_PW"] = "7"


def timeit(B, H, KV, Sq, Sk, w, reps=20):
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B, H, Sq, 128, device=dev, generator=g).bfloat16()
    k = torch.randn(B, KV, Sk, 128, device=dev, generator=g).bfloat16()
    v = torch.randn(B, KV, Sk, 128, device=dev, generator=g).bfloat16()
    o = torch.empty(B, Sq, H * 128, device=dev, dtype=torch.bfloat16)
    args = (q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, KV, Sq, Sk, w, 1 / math.sqrt(128),
            ff.stream_ptr())
    assert f(*args) == 0
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f(*args)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps * 1e3)
    return round(statistics.median(ts), 2)


S = 3000
# KV tiles per unit at 384 units (2 rounds of 256 / 128 units) and 192 units (one round)
for pw in ([] if os.environ.get("BAND_ONLY") else ["7", "0"]):
  os.environ["ACEHIP_ATTN_PW"] = pw
  for B in (1, 2):
    for n in (1, 2, 3, 4, 6, 8, 11):
        print(json.dumps({"kind": "cross", "pw": pw, "B": B, "units": 24 * 8 * B, "tiles": n, "us": timeit(B, 16, 8, S, 64 * n, -1)}),
              flush=True)
os.environ["ACEHIP_ATTN_PW"] = "7"
# band at B = 1..4 (192 / 384 / 576 / 768 units of 6 tile iterations), persistent and one
# workgroup per unit (ACEHIP_ATTN_PERSIST)
for pers in ("1", "0"):
    os.environ["ACEHIP_ATTN_PERSIST"] = pers
    for B in (1, 2, 3, 4):
        print(json.dumps({"kind": "band", "persist": pers, "B": B, "units": 24 * 8 * B,
                          "us": timeit(B, 16, 8, S, S, 128)}), flush=True)
    print(json.dumps({"kind": "band600", "persist": pers, "B": 2, "units": 59 * 8 * 2,
                      "us": timeit(2, 16, 8, 7500, 7500, 128)}), flush=True)
os.environ["ACEHIP_ATTN_PERSIST"] = "1"
# units of one round, sub-chip: S = 128·nq at B = 1 (8·nq units)
for nq in ([] if os.environ.get("BAND_ONLY") else [17, 20, 24]):
    print(json.dumps({"kind": "cross_nq", "units": 8 * nq, "tiles": 6, "us": timeit(1, 16, 8, 128 * nq, 384, -1)}),
          flush=True)
