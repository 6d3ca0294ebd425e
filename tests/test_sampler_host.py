"""CPU check of the sampler HOST logic of ``AceStepDiTBackend.generate_audio``
(schedule, cover-noise truncation, cover -> non-cover switch, CFG interval,
SDE re-noise, turbo table / x0, sft timesteps) against the reference's own
recorded runs — bit-exact.

The three HIP sampler entry points are swapped for the oracle's torch
restatement of the same arithmetic (``oracle/sampler_oracle.py``), so what is
checked here is only the Python control flow around them; the HIP kernels
themselves are checked on the GPU by ``test_gpu_sampler.py`` on the same
recordings."""
import pytest
import torch

import test_gpu_sampler as replay
from oracle import sampler_oracle as so


@pytest.fixture
def torch_kernels(monkeypatch):
    import acehip.dit as dit
    state = {}

    def apg_euler_(vt, xt, ra, guidance, dt, apply_cfg, first_step, out_mode=0):
        B = xt.shape[0]
        if apply_cfg < 0:
            v = vt
        elif apply_cfg == 0:
            v = vt[:B]
        else:
            if first_step:
                state["mom"] = so.Momentum()
            v = so.apg(vt[:B], vt[B:], guidance, state["mom"])
        xt.copy_(v if out_mode == 1 else xt - v * torch.tensor(dt, dtype=xt.dtype))

    def adg_euler_(vt, xt, guidance, sigma, dt, out_mode=0):
        B = xt.shape[0]
        v = so.adg(xt, vt[:B], vt[B:], torch.tensor(sigma, dtype=xt.dtype), guidance)
        xt.copy_(v if out_mode == 1 else xt - v * torch.tensor(dt, dtype=xt.dtype))

    def axpy_(vt, xt, s):
        xt.copy_(xt - vt * torch.tensor(s, dtype=xt.dtype))

    monkeypatch.setattr(dit, "apg_euler_", apg_euler_)
    monkeypatch.setattr(dit, "adg_euler_", adg_euler_)
    monkeypatch.setattr(dit, "axpy_", axpy_)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)


@pytest.mark.parametrize("name", replay.REPLAY)
def test_sampler_host_loop_bit_exact(torch_kernels, monkeypatch, name):
    meta, gd, rt, res, calls, used = replay._replay(torch.device("cpu"), monkeypatch, name)
    assert rt.i == meta["n_calls"] and rt.worst == 0.0
    assert len(used) == (meta.get("n_noise") or 0)
    assert torch.equal(res["target_latents"], gd["target_latents"])


def test_base_ignores_timesteps_host(torch_kernels, monkeypatch):
    meta, gd, rt, res, *_ = replay._replay(torch.device("cpu"), monkeypatch, "base_s8_sh3",
                                           accepts_timesteps=False,
                                           kw_extra={"timesteps": torch.tensor([1.0, 0.5, 0.0])})
    assert rt.i == meta["n_calls"]
    assert torch.equal(res["target_latents"], gd["target_latents"])


def test_sft_detected_from_signature():
    """from_reference_model tells base from sft by generate_audio's signature (sft:1811)."""
    from acehip.dit import takes_timesteps

    class Base:
        def generate_audio(self, text_hidden_states, shift=1.0, **kwargs):
            pass

    class Sft:
        def generate_audio(self, text_hidden_states, shift=1.0, timesteps=None, **kwargs):
            pass
    assert not takes_timesteps(Base()) and takes_timesteps(Sft())
