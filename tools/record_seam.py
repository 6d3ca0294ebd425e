#!/usr/bin/env python3
"""Record the reference's DiT-seam calls (this container only; the reference never travels).

Drives the REFERENCE's own ``ServiceGenerateExecuteMixin._build_service_generate_kwargs`` and
``_execute_service_generate_diffusion`` (``acestep/core/generation/handler/
service_generate_execute.py:62-196``, loaded from ``/root/reference`` with a ``loguru`` stub,
as SURVEY §8c says) on a synthetic payload, with a recording stand-in for ``self.model``.  Every
call the seam makes into the model (``prepare_condition`` at :123, ``generate_audio`` at :194)
is written to ``tests/golden/seam_calls.json`` as a call SPEC:

  * the keyword set, in call order;
  * per tensor keyword: dtype, shape, device type, and where the tensor object came from —
    ``payload:<key>`` (the same object as that payload entry), ``handler:<attr>`` (a handler
    attribute), or ``fresh`` plus a value summary (the attention mask built inside the seam,
    the ``timesteps`` tensor built from the request list);
  * per non-tensor keyword: its value (``seed`` as ``"seed_param"`` when it IS the seed the
    caller passed).

Scenarios: base request (seed list, no ``timesteps``), an sft/turbo request with custom
``timesteps``, and a random-seed request (``_resolve_service_seed_param(None)``).

``tests/test_gpu_integration.py`` rebuilds the kwargs of both calls from this spec (its own
synthetic tensors of the recorded dtypes / shapes, objects shared exactly where the reference
shares them) instead of a hand-written dict; ``tests/test_seam_spec.py`` checks the spec on CPU.
"""
from __future__ import annotations

import contextlib
import importlib.util
import json
import os
import sys
import types

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "tests", "golden", "seam_calls.json")
REF = "/root/reference/acestep/core/generation/handler/service_generate_execute.py"


def _load_mixin():
    if "loguru" not in sys.modules:
        m = types.ModuleType("loguru")

        class _L:
            def __getattr__(self, name):
                return lambda *a, **k: None
        m.logger = _L()
        sys.modules["loguru"] = m
    spec = importlib.util.spec_from_file_location("_ref_service_generate_execute", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.ServiceGenerateExecuteMixin


class RecordingModel:
    def __init__(self):
        self.calls = []

    def prepare_condition(self, **kw):
        self.calls.append(("prepare_condition", kw))
        B, T = kw["src_latents"].shape[:2]
        return torch.zeros(B, 7, 16), torch.ones(B, 7), torch.zeros(B, T, 128)

    def generate_audio(self, **kw):
        self.calls.append(("generate_audio", kw))
        return {"target_latents": torch.zeros_like(kw["src_latents"]), "time_costs": {}}


def _payload(B=2, T=60, Lt=12, Ll=20):
    g = torch.Generator().manual_seed(0)
    return {
        "text_hidden_states": torch.randn(B, Lt, 1024, generator=g).bfloat16(),
        "text_attention_mask": torch.ones(B, Lt, dtype=torch.long),
        "lyric_hidden_states": torch.randn(B, Ll, 1024, generator=g).bfloat16(),
        "lyric_attention_mask": torch.ones(B, Ll, dtype=torch.long),
        "refer_audio_acoustic_hidden_states_packed": torch.randn(B, 750, 64, generator=g).bfloat16(),
        "refer_audio_order_mask": torch.arange(B, dtype=torch.long),
        "src_latents": torch.randn(B, T, 64, generator=g).bfloat16(),
        "chunk_mask": torch.ones(B, T, 64, dtype=torch.bfloat16),
        "is_covers": torch.zeros(B, dtype=torch.long),
        "non_cover_text_hidden_states": None,
        "non_cover_text_attention_masks": None,
        "precomputed_lm_hints_25Hz": None,
    }


def _spec(kw, payload, handler, seed_param):
    out = []
    for name, v in kw.items():
        e = {"name": name}
        if isinstance(v, torch.Tensor):
            e.update(kind="tensor", dtype=str(v.dtype).replace("torch.", ""), shape=list(v.shape),
                     device=v.device.type)
            src = [f"payload:{k}" for k, pv in payload.items() if pv is v]
            if v is handler.silence_latent:
                src.append("handler:silence_latent")
            if src:
                e["source"] = src[0]
            else:
                e["source"] = "fresh"
                e["values"] = v.flatten().tolist() if v.numel() <= 64 else {
                    "all_ones": bool((v == 1).all()), "numel": v.numel()}
        else:
            e["kind"] = "value"
            e["value"] = "seed_param" if (name == "seed" and v is seed_param) else v
        out.append(e)
    return out


def main():
    Mixin = _load_mixin()

    class Host(Mixin):
        def __init__(self):
            self.device = "cpu"
            self.silence_latent = torch.zeros(1, 120, 64, dtype=torch.bfloat16)
            self.use_mlx_dit = False
            self.mlx_decoder = None
            self.model = RecordingModel()

        @contextlib.contextmanager
        def _load_model_context(self, name):
            yield

    scenarios = {
        "base_seed_list": dict(seed_list=[11, 12], timesteps=None, shift=3.0, infer_steps=4),
        "custom_timesteps": dict(seed_list=[5, 6], timesteps=[1.0, 0.75, 0.5, 0.25], shift=1.0, infer_steps=4),
        "random_seed": dict(seed_list=None, timesteps=None, shift=1.0, infer_steps=8),
    }
    rec = {"reference": "acestep/core/generation/handler/service_generate_execute.py:62-196",
           "generator": "tools/record_seam.py", "scenarios": {}}
    for sname, sc in scenarios.items():
        h = Host()
        payload = _payload()
        seed_param = h._resolve_service_seed_param(sc["seed_list"])
        kw = h._build_service_generate_kwargs(
            payload=payload, seed_param=seed_param, infer_steps=sc["infer_steps"], guidance_scale=7.0,
            audio_cover_strength=1.0, cover_noise_strength=0.0, infer_method="ode", use_adg=False,
            cfg_interval_start=0.0, cfg_interval_end=1.0, shift=sc["shift"], timesteps=sc["timesteps"])
        outputs, enc, enc_mask, ctx = h._execute_service_generate_diffusion(
            payload=payload, generate_kwargs=kw, seed_param=seed_param, infer_method="ode", shift=sc["shift"],
            audio_cover_strength=1.0)
        calls = [{"method": m, "kwargs": _spec(k, payload, h, seed_param)} for m, k in h.model.calls]
        # the generate_audio call receives the very dict _build_service_generate_kwargs built
        assert h.model.calls[-1][1].keys() == kw.keys() and all(h.model.calls[-1][1][k] is kw[k] for k in kw)
        rec["scenarios"][sname] = {
            "request": {k: v for k, v in sc.items()},
            "payload": {k: ({"dtype": str(v.dtype).replace("torch.", ""), "shape": list(v.shape)}
                            if isinstance(v, torch.Tensor) else None) for k, v in payload.items()},
            "silence_latent": {"dtype": "bfloat16", "shape": list(h.silence_latent.shape)},
            "calls": calls,
            "returns": {"prepare_condition_outputs_returned": enc is not None and ctx is not None},
        }
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(rec, f, indent=1, sort_keys=False)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
