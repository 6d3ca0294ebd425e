"""CPU restatement of the ACE-Step 1.5 flow-matching samplers — TEST ORACLE ONLY.

Restates ``generate_audio`` of the base/sft model
(``acestep/models/base/modeling_acestep_v15_base.py:1783-1989``, sft adds a
``timesteps`` override ``sft/...:1864-1875``), the turbo model
(``acestep/models/turbo/modeling_acestep_v15_turbo.py:1780-2001``) and APG
guidance (``acestep/models/base/apg_guidance.py:5-56``) on top of an arbitrary
``forward(xt, t_vec) -> vt`` callable, so the same driver can run the CPU DiT
oracle or (in tests) compare against the HIP path step by step.
"""
from __future__ import annotations

from typing import Callable, List, Optional

import torch

Tensor = torch.Tensor

# turbo tables (turbo:1808-1823)
TURBO_VALID_SHIFTS = [1.0, 2.0, 3.0]
TURBO_VALID_TIMESTEPS = [
    1.0, 0.9545454545454546, 0.9333333333333333, 0.9, 0.875,
    0.8571428571428571, 0.8333333333333334, 0.7692307692307693, 0.75,
    0.6666666666666666, 0.6428571428571429, 0.625, 0.5454545454545454,
    0.5, 0.4, 0.375, 0.3, 0.25, 0.2222222222222222, 0.125,
]
TURBO_SHIFT_TIMESTEPS = {
    1.0: [1.0, 0.875, 0.75, 0.625, 0.5, 0.375, 0.25, 0.125],
    2.0: [1.0, 0.9333333333333333, 0.8571428571428571, 0.7692307692307693,
          0.6666666666666666, 0.5454545454545454, 0.4, 0.2222222222222222],
    3.0: [1.0, 0.9545454545454546, 0.9, 0.8333333333333334, 0.75,
          0.6428571428571429, 0.5, 0.3],
}


def base_schedule(infer_steps: int, shift: float, dtype, device="cpu",
                  timesteps: Optional[Tensor] = None) -> Tensor:
    """base:1864-1867 / sft:1866-1875 — linspace and shift in the model dtype."""
    if timesteps is not None:
        return timesteps.to(device=device, dtype=dtype)
    t = torch.linspace(1.0, 0.0, infer_steps + 1, device=device, dtype=dtype)
    if shift != 1.0:
        t = shift * t / (1 + (shift - 1) * t)
    return t


def turbo_schedule_list(shift: float = 3.0, timesteps=None) -> List[float]:
    """turbo:1826-1865 — custom timesteps (trailing zeros stripped, ≤20, mapped
    to the nearest valid value) else the table of the nearest valid shift."""
    sched = None
    if timesteps is not None:
        lst = timesteps.tolist() if isinstance(timesteps, torch.Tensor) else list(timesteps)
        while lst and lst[-1] == 0:
            lst.pop()
        if len(lst) >= 1:
            sched = [min(TURBO_VALID_TIMESTEPS, key=lambda x: abs(x - t)) for t in lst[:20]]
    if sched is None:
        s = min(TURBO_VALID_SHIFTS, key=lambda x: abs(x - shift))
        sched = list(TURBO_SHIFT_TIMESTEPS[s])
    return sched


class Momentum:
    """MomentumBuffer (apg_guidance.py:5-13)."""

    def __init__(self, momentum: float = -0.75):
        self.momentum = momentum
        self.running_average = 0

    def update(self, v: Tensor):
        self.running_average = v + self.momentum * self.running_average


def apg(pred_cond: Tensor, pred_uncond: Tensor, guidance_scale: float,
        mom: Optional[Momentum], dims=(1,), eta: float = 0.0,
        norm_threshold: float = 2.5) -> Tensor:
    """apg_forward + project (apg_guidance.py:16-56): momentum and norm clip in
    the activation dtype, projection in float64."""
    diff = pred_cond - pred_uncond
    if mom is not None:
        mom.update(diff)
        diff = mom.running_average
    dims = list(dims)
    if norm_threshold > 0:
        n = diff.norm(p=2, dim=dims, keepdim=True)
        diff = diff * torch.minimum(torch.ones_like(diff), norm_threshold / n)
    dt = diff.dtype
    v0, v1 = diff.double(), pred_cond.double()
    v1 = torch.nn.functional.normalize(v1, dim=dims)
    par = (v0 * v1).sum(dim=dims, keepdim=True) * v1
    orth = v0 - par
    upd = orth.to(dt) + eta * par.to(dt)
    return pred_cond + (guidance_scale - 1) * upd


def adg(latents: Tensor, cond: Tensor, uncond: Tensor, sigma: Tensor, guidance_scale: float,
        angle_clip: float = 3.14 / 6) -> Tensor:
    """adg_forward (apg_guidance.py:107-180, apply_norm=False, apply_clip=True)
    with its dtype chain: hats in the activation dtype, the angle in float64
    (call_cos_tensor :63-77 on ``.to(float)``), the perpendicular split in
    float32 (compute_perpendicular_component :80-104), the recombination in
    float64, cast back at the end.  Row-local over the channel axis.  The
    reference's ``[N·T,1] × [N,T,C]`` broadcast only works for N = 1; this
    restatement keeps that exact op order (tests use N = 1)."""
    n, t, c = cond.shape
    sigma = sigma.reshape(1, 1, 1).expand(n, 1, 1) if sigma.numel() == 1 else sigma.view(n, 1, 1)
    w = guidance_scale - 1
    w = w * (w > 0) + 1e-3
    ht = latents - sigma * cond
    hu = latents - sigma * uncond
    diff = ht - hu
    a, b = ht.view(-1, c).to(torch.float64), hu.reshape(-1, c).contiguous().to(torch.float64)
    a = a / torch.linalg.norm(a, dim=1, keepdim=True)
    b = b / torch.linalg.norm(b, dim=1, keepdim=True)
    theta = torch.acos(torch.sum(a * b, dim=1, keepdim=True))
    theta_new = torch.clip(w * theta, -angle_clip, angle_clip)
    d32, u32 = diff.view(n * t, c).float(), hu.view(n * t, c).float()
    dot = torch.sum(d32 * u32, dim=1, keepdim=True)
    nsq = torch.sum(u32 * u32, dim=1, keepdim=True)
    perp = (d32 - (dot / (nsq + 1e-8)) * u32).reshape(n, t, c)
    if n == 1:
        cs, sn, st = torch.cos(theta_new), torch.sin(theta_new), torch.sin(theta)
    else:   # per-row generalisation (the reference raises a broadcast error here)
        cs, sn, st = (v.view(n, t, 1) for v in (torch.cos(theta_new), torch.sin(theta_new), torch.sin(theta)))
    v_new = cs * ht
    p_new = perp * sn / st * (st > 1e-3) + perp * w * (st <= 1e-3)
    new = v_new + p_new
    return ((latents - new) / sigma).reshape(n, t, c).to(latents.dtype)


def generate_base(forward: Callable[[Tensor, Tensor], Tensor], noise: Tensor,
                  infer_steps: int, guidance: float = 7.0, shift: float = 1.0,
                  infer_method: str = "ode", cfg_interval_start: float = 0.0,
                  cfg_interval_end: float = 1.0, timesteps: Optional[Tensor] = None,
                  step_hook=None, use_adg: bool = False) -> Tensor:
    """The base/sft step loop (base:1864-1979) with ``forward(x, t_vec)``
    standing in for the decoder call (the batch is doubled for CFG by this
    function, exactly as base:1929).  APG, or ADG with ``use_adg`` (base:1949-1964)."""
    dtype, device = noise.dtype, noise.device
    t = base_schedule(infer_steps, shift, dtype, device, timesteps)
    n_steps = len(t) - 1
    xt = noise
    bsz = xt.shape[0]
    do_cfg = guidance > 1.0
    mom = Momentum()
    for i, (tc, tp) in enumerate(zip(t[:-1], t[1:])):
        x = torch.cat([xt, xt], 0) if do_cfg else xt
        tv = tc * torch.ones((x.shape[0],), device=device, dtype=dtype)
        vt = forward(x, tv)
        if do_cfg:
            cond, uncond = vt.chunk(2)
            if tc >= cfg_interval_start and tc <= cfg_interval_end:
                vt = (adg(xt, cond, uncond, tc, guidance) if use_adg
                      else apg(cond, uncond, guidance, mom, dims=(1,)))
            else:
                vt = cond
        if step_hook is not None:
            step_hook(i, xt, vt)
        if infer_method == "sde":
            tb = tc * torch.ones((bsz,), device=device, dtype=dtype)
            x0 = xt - vt * tb[:, None, None]
            nt = 1.0 - float(i + 1) / n_steps
            xt = nt * torch.randn_like(x0) + (1 - nt) * x0
        else:
            dtv = (tc - tp) * torch.ones((bsz,), device=device, dtype=dtype)[:, None, None]
            xt = xt - vt * dtv
    return xt


def generate_turbo(forward: Callable[[Tensor, Tensor], Tensor], noise: Tensor,
                   shift: float = 3.0, timesteps=None, infer_method: str = "ode") -> Tensor:
    """The turbo step loop (turbo:1941-1991): bf16-rounded table values read
    back with .item(), final step x0 = xt - vt*t, ODE dt in Python double."""
    dtype, device = noise.dtype, noise.device
    sched = torch.tensor(turbo_schedule_list(shift, timesteps), device=device, dtype=dtype)
    n = len(sched)
    xt = noise
    bsz = xt.shape[0]
    for i in range(n):
        tc = sched[i].item()
        tv = tc * torch.ones((bsz,), device=device, dtype=dtype)
        vt = forward(xt, tv)
        if i == n - 1:
            return xt - vt * tv[:, None, None]
        tn = sched[i + 1].item()
        if infer_method == "sde":
            x0 = xt - vt * tv[:, None, None]
            xt = tn * torch.randn_like(x0) + (1 - tn) * x0
        else:
            xt = xt - vt * ((tc - tn) * torch.ones((bsz,), device=device, dtype=dtype)[:, None, None])
    return xt
