"""Rebuild the reference seam's model calls from ``tests/golden/seam_calls.json``.

The fixture was recorded by ``tools/record_seam.py`` from the reference's own
``_build_service_generate_kwargs`` / ``_execute_service_generate_diffusion``
(``service_generate_execute.py:62-196``).  :func:`build_calls` returns the payload and the
``(method, kwargs)`` list a handler makes into ``self.model`` for one request, with synthetic
tensors of the recorded dtypes / shapes and object identity shared exactly as the reference
shares it (the same payload tensor in both calls, the handler's ``silence_latent``, a fresh
all-ones ``attention_mask``, a fresh fp32 ``timesteps`` tensor).
"""
import json
import os

import torch

SPEC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "seam_calls.json")


def load_spec():
    with open(SPEC) as f:
        return json.load(f)


def _dtype(name):
    return getattr(torch, name)


def _payload_tensor(key, dtype, shape, g, dev):
    if key.endswith("attention_mask"):
        t = torch.ones(*shape, dtype=dtype)
        t[-1, shape[1] * 3 // 4:] = 0            # a padded tail on the last item
        return t.to(dev)
    if key == "refer_audio_order_mask":
        return torch.arange(shape[0], dtype=dtype, device=dev)
    if key == "is_covers":
        return torch.zeros(*shape, dtype=dtype, device=dev)
    if key == "chunk_mask":
        return torch.ones(*shape, dtype=dtype, device=dev)
    return torch.randn(*shape, generator=g).to(dev, dtype)


def build_calls(scenario, dev, seed_param, seed=17):
    sc = load_spec()["scenarios"][scenario]
    g = torch.Generator(device="cpu").manual_seed(seed)
    payload = {k: (None if v is None else _payload_tensor(k, _dtype(v["dtype"]), v["shape"], g, dev))
               for k, v in sc["payload"].items()}
    sl = sc["silence_latent"]
    silence = torch.randn(*sl["shape"], generator=g).to(dev, _dtype(sl["dtype"]))
    calls = []
    for c in sc["calls"]:
        kw = {}
        for e in c["kwargs"]:
            if e["kind"] == "value":
                kw[e["name"]] = seed_param if e["value"] == "seed_param" else e["value"]
                continue
            src = e["source"]
            if src.startswith("payload:"):
                t = payload[src.split(":", 1)[1]]
            elif src == "handler:silence_latent":
                t = silence
            else:                                   # fresh: built inside the seam
                vals = e["values"]
                if isinstance(vals, dict):
                    assert vals["all_ones"]
                    t = torch.ones(*e["shape"], dtype=_dtype(e["dtype"]), device=dev)
                else:
                    t = torch.tensor(vals, dtype=_dtype(e["dtype"]), device=dev).reshape(e["shape"])
            assert list(t.shape) == e["shape"] and t.dtype == _dtype(e["dtype"]), e["name"]
            kw[e["name"]] = t
        calls.append((c["method"], kw))
    return payload, silence, calls
