#!/usr/bin/env python3
"""Full attention at 240 s (Bc = 2, S = 3000, 384 units on 256 CUs): where the time goes —
one round (B = 1), two whole rounds (no tail split, ACEHIP_ATTN_CUS = 384), the default
tail split (second round split over 2 KV ranges + merge), and forced 3/4-way tails."""
import json, math, os, statistics, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
import torch  # noqa: E402
from acehip import _ffi as ff  # noqa: E402
dev = torch.device("cuda:0")
f = ff.lib().acehip_attention_bf16


def timeit(B, S, w=-1, reps=20):
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B, 16, S, 128, device=dev, generator=g).bfloat16()
    k = torch.randn(B, 8, S, 128, device=dev, generator=g).bfloat16()
    v = torch.randn(B, 8, S, 128, device=dev, generator=g).bfloat16()
    o = torch.empty(B, S, 16 * 128, device=dev, dtype=torch.bfloat16)
    args = (q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, 16, 8, S, S, w, 1 / math.sqrt(128),
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


for pw in ("0", "1"):
    os.environ["ACEHIP_ATTN_PW"] = pw
    for name, B, cus in (("one_round_B1", 1, ""), ("default_split", 2, ""), ("no_split_2rounds", 2, "384"),
                         ("split4_tail64", 2, "320")):
        if cus:
            os.environ["ACEHIP_ATTN_CUS"] = cus
        else:
            os.environ.pop("ACEHIP_ATTN_CUS", None)
        print(json.dumps({"pw": pw, "case": name, "B": B, "plan_cus": cus or 256, "us": timeit(B, 3000)}), flush=True)
        if name == "default_split":
            for _ in range(3):
                os.environ["ACEHIP_ATTN_DBG"] = "1"
                a = timeit(B, 3000)
                os.environ.pop("ACEHIP_ATTN_DBG")
                b = timeit(B, 3000)
                print(json.dumps({"pw": pw, "case": "no_handoff(wrong results) vs default", "us": [a, b]}), flush=True)
os.environ.pop("ACEHIP_ATTN_CUS", None)
