"""GPU parity of every sampler branch of ``generate_audio`` against the
reference's own recorded runs (``tools/make_golden.py``: the reference
``generate_audio`` driven by a deterministic stand-in decoder that records
every call's x, t, encoder states, context and output, plus every unseeded
``randn_like`` draw of the SDE branch).

The drop-in ``AceStepDiTBackend.generate_audio`` runs with a replay runtime in
place of the DiT: each forward returns the reference's recorded decoder output
for that call, so what is checked is everything around the decoder — the
schedule, cover-noise truncation, the cover -> non-cover switch, CFG + APG /
ADG, the Euler / x0 updates and the SDE re-noise — on the HIP sampler kernels
(``acehip_sampler_apg_euler`` / ``_adg_euler`` / ``_axpy``), call by call.

Branches (reference lines):
  base/sft ODE + APG            base:1915-1979, apg_guidance.py:5-56
  cover-noise truncation        base:1879-1902, turbo:1922-1936
  cover -> non-cover switch     base:1836-1856,1916-1927, turbo:1892-1956
  SDE x0 + re-noise             base:1968-1973, turbo:1980-1984
  turbo table / x0 final step   turbo:1941-1991
  sft custom timesteps          sft:1866-1868 (base ignores them, base:1812)
"""
import pytest
import torch

from conftest import golden_manifest, load_golden, rel_l2

from acehip.config import DiTConfig
from acehip.weights import synth_null_condition
from oracle import sampler_oracle

pytestmark = pytest.mark.gpu

# the recorded trajectories are bf16 (or fp32) end to end; the HIP kernels reduce in a
# different order than torch (fp32 / fp64), so allow a few ulps of drift of the storage type
TOL_STEP = 5e-3
TOL_STEP_FP32 = 1e-5

TURBO_CUSTOM_TIMESTEPS = [0.97, 0.76, 0.5, 0.26, 0.0]     # make_golden.py turbo_custom


class ReplayRuntime:
    """Stands in for DiTRuntime: forward() returns the reference's recorded decoder
    output of the same call after checking what the backend fed it."""

    def __init__(self, gd, n_calls, device, tol=TOL_STEP):
        self.gd, self.n, self.device, self.i = gd, n_calls, device, 0
        self.tol = tol
        self.enc = None
        self.worst = 0.0
        self.conditions = 0

    def set_condition(self, enc):
        self.enc = enc.clone()
        self.conditions += 1

    def set_uniform_rows(self, first_row):
        pass

    def forward(self, xt, ctx, t, t_r=None, out=None):
        i = self.i
        assert i < self.n, "more decoder calls than the reference made"
        self.i += 1
        gd = self.gd
        B = xt.shape[0]
        self.worst = max(self.worst, rel_l2(xt.float().cpu(), gd[f"x_{i}"][:B].float()))
        assert self.worst < self.tol, (i, self.worst)
        # the timestep is the reference's bf16 value
        assert float(t.reshape(-1)[0]) == float(gd[f"t_{i}"][0].float()), (i, float(t[0]), gd[f"t_{i}"])
        # condition (incl. the CFG null rows and the non-cover switch) and context exact
        enc_ref = gd.get(f"enc_{i}", gd["enc"])
        assert torch.equal(self.enc.cpu(), enc_ref), i
        ctx_ref = gd.get(f"ctx_{i}", gd["ctx"])
        assert torch.equal(ctx.cpu(), ctx_ref[:B]), i
        return gd[f"vt_{i}"].to(self.device).contiguous()


def _cpu_noise(shape, device, dtype, seed):
    """prepare_noise (base:1733-1770) on the CPU generator the fixtures were made with."""
    return sampler_oracle_prepare_noise(shape, dtype, seed).to(device)


def sampler_oracle_prepare_noise(shape, dtype, seed):
    B, T, C = shape
    if isinstance(seed, list):
        return torch.cat([torch.randn(1, T, C, generator=torch.Generator().manual_seed(int(s)), dtype=dtype)
                          for s in seed], 0)
    return torch.randn(shape, generator=torch.Generator().manual_seed(int(seed)), dtype=dtype)


REPLAY = ["base_s8_sh3", "base_s27_sh3", "base_s60_sh3", "base_s10_sh1_interval", "base_s8_adg",
          "turbo_sh3", "turbo_sh2", "turbo_custom",
          "base_s8_cover", "base_s8_acs", "base_s8_sde", "base_s10_cover_acs_sde",
          "turbo_cover_acs", "turbo_sde", "sft_timesteps",
          # the fp32 parity mode: same chains, no bf16 rounding
          "base_s8_nocfg_fp32", "base_s8_sh3_fp32", "base_s8_adg_fp32", "turbo_sh3_fp32"]


def _dtype(meta):
    return torch.float32 if "float32" in meta["dtype"] else torch.bfloat16


def _replay(gpu_device, monkeypatch, name, accepts_timesteps=None, kw_extra=None):
    import acehip.dit as dit
    meta = golden_manifest()["sampler"][name]
    kw = dict(meta["kwargs"])
    gd = load_golden("sampler_" + name)
    B, T = meta["B"], meta["T"]
    turbo = meta["variant"] == "turbo"
    if name == "turbo_custom":
        kw["timesteps"] = torch.tensor(TURBO_CUSTOM_TIMESTEPS)
    elif isinstance(kw.get("timesteps"), list):
        # the handler hands custom timesteps over as an fp32 device tensor
        # (service_generate_execute.py:103-104)
        kw["timesteps"] = torch.tensor(kw["timesteps"], dtype=torch.float32, device=gpu_device)
    kw.update(kw_extra or {})
    if accepts_timesteps is None:
        accepts_timesteps = meta["variant"] in ("sft", "turbo")
    dtype = _dtype(meta)
    rt = ReplayRuntime(gd, meta["n_calls"], gpu_device, TOL_STEP_FP32 if dtype == torch.float32 else TOL_STEP)
    cfg = DiTConfig.tiny(layers=1)
    null = synth_null_condition(cfg, seed=7).to(dtype)
    nb = B

    # prepare_condition stand-in: the reference's recorded encoder states / context of the
    # cover condition first, then (audio_cover_strength < 1) of the non-cover condition
    first = gd.get("enc_0", gd["enc"])
    switch = next((i for i in range(meta["n_calls"]) if f"enc_{i}" in gd and not torch.equal(gd[f"enc_{i}"], first)), None)
    conds = [(first[:nb], gd.get("ctx_0", gd["ctx"])[:nb])]
    if switch is not None:
        conds.append((gd[f"enc_{switch}"][:nb], gd[f"ctx_{switch}"][:nb]))
    calls = []

    def prepare_condition(**k):
        e, c = conds[len(calls)]
        calls.append(k)
        return e.to(gpu_device), None, c.to(gpu_device)

    be = dit.AceStepDiTBackend(rt, null, is_turbo=turbo, prepare_condition=prepare_condition,
                               accepts_timesteps=accepts_timesteps, dtype=dtype)
    monkeypatch.setattr(dit, "prepare_noise", _cpu_noise)
    draws = [gd[f"noise_{i}"] for i in range(meta.get("n_noise") or 0)]
    used = []

    def randn_like(x, *a, **k):
        n = draws[len(used)]
        used.append(1)
        assert n.shape == x.shape
        return n.to(device=x.device, dtype=x.dtype)
    monkeypatch.setattr(torch, "randn_like", randn_like)
    src = gd["src_latents"][:B].to(gpu_device) if "src_latents" in gd else torch.zeros(B, T, 64)
    sil = gd["silence_latent"].to(gpu_device) if "silence_latent" in gd else torch.zeros(1, T, 64)
    res = be.generate_audio(text_hidden_states=None, text_attention_mask=None, lyric_hidden_states=None,
                            lyric_attention_mask=None, refer_audio_acoustic_hidden_states_packed=None,
                            refer_audio_order_mask=None, src_latents=src.to(dtype),
                            chunk_masks=torch.ones(B, T, 64, dtype=dtype, device=gpu_device),
                            is_covers=torch.zeros(B, dtype=torch.long, device=gpu_device),
                            silence_latent=sil.to(dtype), seed=list(range(B)), **kw)
    torch.cuda.synchronize()
    return meta, gd, rt, res, calls, used


@pytest.mark.parametrize("name", REPLAY)
def test_generate_audio_replays_reference(gpu_device, monkeypatch, name):
    meta, gd, rt, res, calls, used = _replay(gpu_device, monkeypatch, name)
    assert rt.i == meta["n_calls"], (rt.i, meta["n_calls"])               # same number of decoder calls
    assert len(used) == (meta.get("n_noise") or 0)                         # same number of SDE draws
    out = res["target_latents"]
    assert out.shape == gd["target_latents"].shape and out.dtype == gd["target_latents"].dtype
    tol = TOL_STEP_FP32 if out.dtype == torch.float32 else TOL_STEP
    assert rel_l2(out.float().cpu(), gd["target_latents"].float()) < tol, rel_l2(
        out.float().cpu(), gd["target_latents"].float())
    acs = meta["kwargs"].get("audio_cover_strength", 1.0)
    assert len(calls) == (2 if acs < 1.0 else 1)                            # non-cover prepare_condition
    assert set(res["time_costs"]) >= {"encoder_time_cost", "diffusion_time_cost",
                                      "diffusion_per_step_time_cost", "total_time_cost"}


def test_base_ignores_timesteps(gpu_device, monkeypatch):
    """base has no ``timesteps`` parameter (base:1783-1813, swallowed by **kwargs): a base
    backend given custom timesteps runs the linspace+shift schedule — the base_s8_sh3
    recording replays unchanged."""
    meta, gd, rt, res, *_ = _replay(gpu_device, monkeypatch, "base_s8_sh3", accepts_timesteps=False,
                                    kw_extra={"timesteps": torch.tensor([1.0, 0.5, 0.0], device=gpu_device)})
    assert rt.i == meta["n_calls"]
    assert rel_l2(res["target_latents"].float().cpu(), gd["target_latents"].float()) < TOL_STEP


def test_sft_honours_timesteps_schedule(gpu_device):
    """sft (sft:1866-1868): the schedule is the given tensor cast to the model dtype —
    bit-exact against the oracle's restatement."""
    from acehip.dit import base_schedule
    ts = torch.tensor([1.0, 0.9, 0.7, 0.5, 0.3, 0.1, 0.0], dtype=torch.float32)
    dev = base_schedule(99, 3.0, gpu_device, torch.bfloat16, ts.to(gpu_device)).cpu()
    ref = sampler_oracle.base_schedule(99, 3.0, torch.bfloat16, timesteps=ts)
    assert torch.equal(dev.view(torch.int16), ref.view(torch.int16))
