"""DiT runtime handle + the ``generate_audio`` drop-in backend.

``AceStepDiTBackend.generate_audio(**kwargs)`` keeps the contract of the
reference ``AceStepConditionGenerationModel.generate_audio`` — base/sft
(``acestep/models/base/modeling_acestep_v15_base.py:1783-1989``, sft's
``timesteps`` override ``sft/...:1864-1875``) and turbo
(``acestep/models/turbo/modeling_acestep_v15_turbo.py:1780-2001``) — and
returns ``{"target_latents", "time_costs"}``, so the reference caller
(``acestep/core/generation/handler/service_generate_execute.py:191,194``)
needs no change.

Host plumbing stays in PyTorch exactly where the reference's own semantics
live in PyTorch: the timestep schedule (linspace/shift in the model dtype on
the model device), per-seed Philox noise (``prepare_noise``, base:1733-1770),
and the unseeded SDE re-noise.  Every DiT forward, the CFG/APG guidance and
the Euler update run in libacehip's HIP kernels; there is no CPU or eager
fallback (``_ffi.lib()`` raises if the library is absent).
"""
from __future__ import annotations

import inspect
import os
import math
import time
from typing import Dict, List, Optional, Union

import torch

from . import _ffi
from .config import DiTConfig
from ._ffi import ACEHIP_BF16, ACEHIP_F32, check, lib, ptr, shape_arg, stream_ptr

# turbo tables (turbo:1808-1823)
_TURBO_VALID_SHIFTS = [1.0, 2.0, 3.0]
_TURBO_VALID_T = [
    1.0, 0.9545454545454546, 0.9333333333333333, 0.9, 0.875, 0.8571428571428571,
    0.8333333333333334, 0.7692307692307693, 0.75, 0.6666666666666666, 0.6428571428571429,
    0.625, 0.5454545454545454, 0.5, 0.4, 0.375, 0.3, 0.25, 0.2222222222222222, 0.125,
]
_TURBO_TABLE = {
    1.0: [1.0, 0.875, 0.75, 0.625, 0.5, 0.375, 0.25, 0.125],
    2.0: [1.0, 0.9333333333333333, 0.8571428571428571, 0.7692307692307693,
          0.6666666666666666, 0.5454545454545454, 0.4, 0.2222222222222222],
    3.0: [1.0, 0.9545454545454546, 0.9, 0.8333333333333334, 0.75, 0.6428571428571429, 0.5, 0.3],
}


class DiTRuntime:
    """One ``acehip_dit`` handle: packed weights, cross-K/V cache, workspace."""

    def __init__(self, cfg: DiTConfig, device: Union[int, torch.device] = 0, max_S: int = 7500,
                 max_Bc: int = 2, max_Lenc: int = 1024, dtype: torch.dtype = torch.bfloat16):
        """dtype bfloat16: the production path; float32: the fp32 parity mode (SURVEY
        §8c(iii) — the reference's fp32 forward, fp32 weights / activations / accumulation)."""
        if dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("DiTRuntime: dtype must be torch.bfloat16 or torch.float32")
        self.cfg = cfg
        self.dtype = dtype
        self.device = torch.device("cuda", device if isinstance(device, int) else device.index or 0)
        self.max_S, self.max_Bc, self.max_Lenc = max_S, max_Bc, max_Lenc
        sl = (_ffi.c_uint8 * cfg.num_hidden_layers)(
            *[1 if cfg.is_sliding(i) else 0 for i in range(cfg.num_hidden_layers)])
        self._sliding = sl
        c = _ffi.DiTCfg(hidden=cfg.hidden_size, intermediate=cfg.intermediate_size,
                        heads=cfg.num_attention_heads, kv_heads=cfg.num_key_value_heads,
                        head_dim=cfg.head_dim, layers=cfg.num_hidden_layers,
                        window=cfg.sliding_window, patch=cfg.patch_size,
                        in_channels=cfg.in_channels, out_channels=cfg.audio_acoustic_hidden_dim,
                        eps=cfg.rms_norm_eps, rope_theta=cfg.rope_theta, max_S=max_S,
                        max_Bc=max_Bc, max_Lenc=max_Lenc,
                        sliding=_ffi.ctypes.cast(sl, _ffi.POINTER(_ffi.c_uint8)),
                        fp32=1 if dtype == torch.float32 else 0)
        h = _ffi.c_void_p()
        check(lib().acehip_dit_create(self.device.index, _ffi.ctypes.byref(c), _ffi.ctypes.byref(h)),
              "dit_create")
        self.h = h
        self.Bc = None
        self.Lenc = None

    # -- weights -------------------------------------------------------------
    def set_weight(self, name: str, t: torch.Tensor):
        t = t.detach().contiguous()
        if t.dtype not in (torch.float32, torch.bfloat16):
            t = t.float()
        dt = ACEHIP_F32 if t.dtype == torch.float32 else ACEHIP_BF16
        on_dev = 1 if t.is_cuda else 0
        check(lib().acehip_dit_set_weight(self.h, name.encode(), ptr(t), dt, t.dim(),
                                          shape_arg(tuple(t.shape)), on_dev), f"set_weight({name})")

    def load(self, weights: Dict[str, torch.Tensor]):
        """Reference state-dict names (with or without the ``decoder.`` prefix)."""
        # the reference's own fp32 constants for the sinusoid / RoPE (base:239-241,
        # Qwen3RotaryEmbedding init) — computed with torch exactly as it does
        freqs = torch.exp(-math.log(10000) * torch.arange(0, 128, dtype=torch.float32) / 128)
        self.set_weight("_timestep_freqs", freqs)
        hd = self.cfg.head_dim
        inv = 1.0 / (self.cfg.rope_theta ** (torch.arange(0, hd, 2, dtype=torch.float) / hd))
        self.set_weight("_rope_inv_freq", inv)
        for k, v in weights.items():
            if k.startswith("decoder."):
                k = k[len("decoder."):]
            if k.startswith("rotary_emb.") or k == "null_condition_emb":
                continue
            self.set_weight(k, v)
        check(lib().acehip_dit_finalize(self.h), "dit_finalize")

    # -- compute -------------------------------------------------------------
    def set_condition(self, enc: torch.Tensor):
        """enc: [Bc, Lenc, D] on the device (pre condition_embedder), cast to the runtime dtype."""
        enc = enc.to(device=self.device, dtype=self.dtype).contiguous()
        Bc, Lenc, _ = enc.shape
        check(lib().acehip_dit_set_condition(self.h, ptr(enc), Bc, Lenc, stream_ptr()), "set_condition")
        self._enc_keepalive = enc
        self.Bc, self.Lenc = Bc, Lenc

    def set_uniform_rows(self, first_row: int):
        """Rows [first_row, Bc) of the condition are one vector repeated (CFG null rows):
        their cross-attention is computed in closed form (acehip_dit_set_uniform_rows)."""
        check(lib().acehip_dit_set_uniform_rows(self.h, int(first_row), stream_ptr()), "set_uniform_rows")

    def forward(self, xt: torch.Tensor, ctx: torch.Tensor, t: torch.Tensor,
                t_r: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One decoder forward.  xt [Bx,T,64], ctx [Bx,T,128] in the runtime dtype; t/t_r:
        fp32 device tensors of 1 (broadcast) or Bc elements.  Returns vt [Bc,T,64]."""
        Bx, T, _ = xt.shape
        Bc = self.Bc
        assert Bc is not None, "set_condition first"
        assert xt.dtype == self.dtype and ctx.dtype == self.dtype, (xt.dtype, ctx.dtype, self.dtype)
        assert xt.is_contiguous() and ctx.is_contiguous() and ctx.shape[:2] == xt.shape[:2]
        if t_r is None:
            t_r = t
        stride = 0 if t.numel() == 1 else 1
        if out is None:
            out = torch.empty(Bc, T, 64, device=xt.device, dtype=self.dtype)
        assert out.dtype == self.dtype and out.is_contiguous()
        dt = ACEHIP_F32 if self.dtype == torch.float32 else ACEHIP_BF16
        check(lib().acehip_dit_forward(self.h, ptr(xt), ptr(ctx), Bx, ptr(t), ptr(t_r), stride, Bc, T, dt,
                                       ptr(out), stream_ptr()), "dit_forward")
        return out

    def set_timesteps(self, t: torch.Tensor, t_r: Optional[torch.Tensor] = None):
        """Timestep MLPs of a whole schedule (one broadcast t per step, fp32 device tensor of
        n steps); forward_step(i) then runs step i without re-reading the MLP weights."""
        t = t.float().contiguous()
        t_r = t if t_r is None else t_r.float().contiguous()
        assert t.dim() == 1 and t_r.shape == t.shape
        self._ts = (t, t_r)          # keep the arrays alive while the kernels read them
        check(lib().acehip_dit_set_timesteps(self.h, ptr(t), ptr(t_r), t.numel(), stream_ptr()), "dit_set_timesteps")

    def forward_step(self, xt: torch.Tensor, ctx: torch.Tensor, step: int,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """forward(xt, ctx, t[step]) of the set_timesteps schedule (bit-identical, bf16)."""
        Bx, T, _ = xt.shape
        Bc = self.Bc
        assert Bc is not None, "set_condition first"
        assert xt.dtype == self.dtype == ctx.dtype == torch.bfloat16
        assert xt.is_contiguous() and ctx.is_contiguous() and ctx.shape[:2] == xt.shape[:2]
        if out is None:
            out = torch.empty(Bc, T, 64, device=xt.device, dtype=self.dtype)
        check(lib().acehip_dit_forward_step(self.h, ptr(xt), ptr(ctx), Bx, int(step), Bc, T, ACEHIP_BF16,
                                            ptr(out), stream_ptr()), "dit_forward_step")
        return out

    def use_graph(self, enable: bool = True):
        """Replay the layer stack of every forward as one captured HIP graph (default off: measured neutral)."""
        check(lib().acehip_dit_set_graph(self.h, 1 if enable else 0), "dit_set_graph")

    PROFILE_KINDS = ["gemm_swiglu", "gemm_down", "gemm_qkv", "gemm_o", "attn_full", "attn_band",
                     "attn_cross"]

    def profile(self, enable: bool = True, kinds=None):
        """Record HIP events around the listed kernel families (default: all)."""
        mask = 0x7f if kinds is None else sum(1 << self.PROFILE_KINDS.index(k) for k in kinds)
        check(lib().acehip_dit_profile_kinds(self.h, mask), "dit_profile_kinds")
        check(lib().acehip_dit_profile(self.h, 1 if enable else 0), "dit_profile")

    def profile_read(self) -> Dict[str, tuple]:
        """{kind: (launches, total_ms)} — call after synchronising the stream."""
        out = {}
        for i, k in enumerate(self.PROFILE_KINDS):
            n, ms = _ffi.c_int(), _ffi.c_float()
            check(lib().acehip_dit_profile_read(self.h, i, _ffi.ctypes.byref(n), _ffi.ctypes.byref(ms)),
                  "dit_profile_read")
            out[k] = (n.value, ms.value)
        return out

    def close(self):
        if getattr(self, "h", None):
            lib().acehip_dit_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _same_dtype(*ts):
    d = ts[0].dtype
    assert all(t is None or (t.dtype == d and t.is_contiguous()) for t in ts), [t.dtype for t in ts if t is not None]
    return _ffi.dtype_code(ts[0])


def apg_euler_(vt, xt, ra, guidance, dt, apply_cfg, first_step, out_mode=0):
    """Fused CFG split + APG + Euler (in place on xt).  vt [2B|B, T, 64]; bf16 or fp32."""
    B, T, C = xt.shape
    dt_code = _same_dtype(xt, vt, ra)
    check(lib().acehip_sampler_apg_euler(ptr(vt), ptr(xt), ptr(ra), B, T, C, float(guidance),
                                         float(dt), int(apply_cfg), int(first_step), int(out_mode), dt_code,
                                         stream_ptr()), "sampler_apg_euler")


def adg_euler_(vt, xt, guidance, sigma, dt, out_mode=0):
    """Fused CFG split + ADG + Euler (in place on xt).  vt [2B, T, 64]; with
    out_mode=1 xt must hold the latents on entry and receives the guided v."""
    B, T, C = xt.shape
    dt_code = _same_dtype(xt, vt)
    check(lib().acehip_sampler_adg_euler(ptr(vt), ptr(xt), B, T, C, float(guidance), float(sigma),
                                         float(dt), int(out_mode), dt_code, stream_ptr()), "sampler_adg_euler")


def axpy_(vt, xt, s):
    """xt = xt − vt·s in place, each op rounded to the storage dtype."""
    dt_code = _same_dtype(xt, vt)
    check(lib().acehip_sampler_axpy(ptr(vt), ptr(xt), xt.numel(), float(s), dt_code, stream_ptr()), "axpy")


def prepare_noise(shape, device, dtype, seed):
    """prepare_noise (base:1733-1770): per-seed device generators."""
    B, T, C = shape
    if seed is None:
        return torch.randn(shape, device=device, dtype=dtype)
    if isinstance(seed, list):
        out = []
        for s in seed:
            if s is None or s < 0:
                out.append(torch.randn(1, T, C, device=device, dtype=dtype))
            else:
                g = torch.Generator(device=device).manual_seed(int(s))
                out.append(torch.randn(1, T, C, generator=g, device=device, dtype=dtype))
        return torch.cat(out, 0)
    g = torch.Generator(device=device).manual_seed(int(seed))
    return torch.randn(shape, generator=g, device=device, dtype=dtype)


def base_schedule(infer_steps, shift, device, dtype, timesteps=None):
    """base:1864-1867 / sft:1866-1875: linspace + shift in the model dtype on the
    model device (torch itself, so the values are the reference's bit for bit)."""
    if timesteps is not None:
        return timesteps.to(device=device, dtype=dtype)
    t = torch.linspace(1.0, 0.0, infer_steps + 1, device=device, dtype=dtype)
    if shift != 1.0:
        t = shift * t / (1 + (shift - 1) * t)
    return t


def turbo_schedule(shift=3.0, timesteps=None) -> List[float]:
    """turbo:1826-1865 (custom timesteps mapped to the 20 valid values, else the
    table of the nearest valid shift)."""
    sched = None
    if timesteps is not None:
        lst = timesteps.tolist() if isinstance(timesteps, torch.Tensor) else list(timesteps)
        while lst and lst[-1] == 0:
            lst.pop()
        if lst:
            sched = [min(_TURBO_VALID_T, key=lambda x: abs(x - t)) for t in lst[:20]]
    if sched is None:
        sched = list(_TURBO_TABLE[min(_TURBO_VALID_SHIFTS, key=lambda x: abs(x - shift))])
    return sched


def takes_timesteps(model) -> bool:
    """base vs sft share one config; they are told apart by ``generate_audio``'s
    signature: sft declares ``timesteps`` (sft:1811), base swallows it in ``**kwargs``."""
    try:
        return "timesteps" in inspect.signature(model.generate_audio).parameters
    except (TypeError, ValueError):
        return False


class AceStepDiTBackend:
    """Drop-in for ``AceStepConditionGenerationModel.generate_audio``."""

    def __init__(self, runtime: DiTRuntime, null_condition_emb: torch.Tensor, is_turbo: bool = False,
                 prepare_condition=None, dtype=torch.bfloat16, accepts_timesteps: Optional[bool] = None):
        self.rt = runtime
        self.device = runtime.device
        if getattr(runtime, "dtype", dtype) != dtype:
            raise ValueError(f"AceStepDiTBackend: runtime dtype {runtime.dtype} != {dtype}")
        self.dtype = dtype          # bf16: production; fp32: the parity mode (DiTRuntime(dtype=fp32))
        self.null = null_condition_emb.detach().to(self.device, dtype)
        self.is_turbo = is_turbo
        # custom ``timesteps``: the turbo (turbo:1803,1828-1857) and sft (sft:1811,1866-1868)
        # samplers honour them; base has no such parameter and swallows it in **kwargs
        # (base:1812), so a base checkpoint ignores it.  None = the turbo default (base).
        self.accepts_timesteps = is_turbo if accepts_timesteps is None else bool(accepts_timesteps)
        self.prepare_condition = prepare_condition
        self.uniform_null = True     # closed-form cross-attention for the CFG null rows

    @classmethod
    def from_reference_model(cls, model, max_seconds: float = 600.0, max_batch: int = 8,
                             max_Lenc: int = 2048):
        """Build from a loaded reference ``AceStepConditionGenerationModel``
        (weights exported from ``model.decoder.state_dict()`` like the MLX
        precedent ``acestep/models/mlx/dit_convert.py:11-66``)."""
        c = model.config
        cfg = DiTConfig(hidden_size=c.hidden_size, intermediate_size=c.intermediate_size,
                        num_hidden_layers=c.num_hidden_layers, num_attention_heads=c.num_attention_heads,
                        num_key_value_heads=c.num_key_value_heads, head_dim=c.head_dim,
                        sliding_window=c.sliding_window, patch_size=c.patch_size,
                        in_channels=c.in_channels, audio_acoustic_hidden_dim=c.audio_acoustic_hidden_dim,
                        rms_norm_eps=c.rms_norm_eps, rope_theta=float(getattr(c, "rope_theta", 1e6)),
                        layer_types=list(c.layer_types))
        dev = next(model.parameters()).device
        max_S = int(max_seconds * 25 + 1) // 2 + 1
        dtype = next(model.parameters()).dtype
        rt = DiTRuntime(cfg, dev.index or 0, max_S=max_S, max_Bc=2 * max_batch, max_Lenc=max_Lenc,
                        dtype=torch.float32 if dtype == torch.float32 else torch.bfloat16)
        rt.load(model.decoder.state_dict())
        turbo = bool(getattr(c, "is_turbo", False)) or getattr(c, "model_version", "") == "turbo"
        return cls(rt, model.null_condition_emb, is_turbo=turbo,
                   prepare_condition=model.prepare_condition, dtype=rt.dtype,
                   accepts_timesteps=turbo or takes_timesteps(model))

    # ------------------------------------------------------------------ API --
    def _condition(self, kw):
        if kw.get("encoder_hidden_states") is not None:
            return kw["encoder_hidden_states"], kw.get("encoder_attention_mask"), kw["context_latents"]
        if self.prepare_condition is None:
            raise RuntimeError("acehip: pass encoder_hidden_states/context_latents or a prepare_condition")
        src = kw["src_latents"]
        am = kw.get("attention_mask")
        if am is None:
            am = torch.ones(src.shape[0], src.shape[1], device=src.device, dtype=src.dtype)
        return self.prepare_condition(
            text_hidden_states=kw["text_hidden_states"], text_attention_mask=kw["text_attention_mask"],
            lyric_hidden_states=kw["lyric_hidden_states"], lyric_attention_mask=kw["lyric_attention_mask"],
            refer_audio_acoustic_hidden_states_packed=kw["refer_audio_acoustic_hidden_states_packed"],
            refer_audio_order_mask=kw["refer_audio_order_mask"], hidden_states=src, attention_mask=am,
            silence_latent=kw.get("silence_latent"), src_latents=src, chunk_masks=kw["chunk_masks"],
            is_covers=kw["is_covers"], precomputed_lm_hints_25Hz=kw.get("precomputed_lm_hints_25Hz"),
            audio_codes=kw.get("audio_codes"))

    def _non_cover_condition(self, kw, ctx):
        if self.prepare_condition is None:
            raise RuntimeError("acehip: audio_cover_strength < 1 needs prepare_condition")
        src = kw["src_latents"]
        sil = kw["silence_latent"][:, : src.shape[1], :].expand(src.shape[0], -1, -1)
        am = kw.get("attention_mask")
        if am is None:
            am = torch.ones(src.shape[0], src.shape[1], device=src.device, dtype=src.dtype)
        is_covers = kw["is_covers"]
        return self.prepare_condition(
            text_hidden_states=kw.get("non_cover_text_hidden_states"),
            text_attention_mask=kw.get("non_cover_text_attention_mask"),
            lyric_hidden_states=kw["lyric_hidden_states"], lyric_attention_mask=kw["lyric_attention_mask"],
            refer_audio_acoustic_hidden_states_packed=kw["refer_audio_acoustic_hidden_states_packed"],
            refer_audio_order_mask=kw["refer_audio_order_mask"], hidden_states=sil, attention_mask=am,
            silence_latent=kw["silence_latent"], src_latents=sil, chunk_masks=kw["chunk_masks"],
            is_covers=torch.zeros_like(is_covers), precomputed_lm_hints_25Hz=None, audio_codes=None)

    def generate_audio(self, **kw) -> Dict:
        t0 = time.time()
        enc, _enc_mask, ctx = self._condition(kw)
        enc_nc = ctx_nc = None
        acs = float(kw.get("audio_cover_strength", 1.0))
        if acs < 1.0:
            if kw.get("_non_cover") is not None:      # conditioned upstream (SongParallelPipeline)
                enc_nc, ctx_nc = kw["_non_cover"]
            else:
                enc_nc, _, ctx_nc = self._non_cover_condition(kw, ctx)
        dtype, device = self.dtype, self.device
        ctx = ctx.to(device=device, dtype=dtype).contiguous()
        enc = enc.to(device=device, dtype=dtype)
        t1 = time.time()
        costs = {"encoder_time_cost": t1 - t0}
        if self.is_turbo:
            xt, n = self._turbo_loop(kw, enc, ctx, enc_nc, ctx_nc, acs)
        else:
            xt, n = self._base_loop(kw, enc, ctx, enc_nc, ctx_nc, acs)
        torch.cuda.synchronize(device)
        t2 = time.time()
        costs["diffusion_time_cost"] = t2 - t1
        costs["diffusion_per_step_time_cost"] = (t2 - t1) / max(n, 1)
        costs["total_time_cost"] = t2 - t0
        return {"target_latents": xt, "time_costs": costs}

    def _noise(self, kw, shape):
        """prepare_noise (base:1733-1770), or the ``_noise`` rows a song-parallel caller drew
        for the whole batch on rank 0 (so an int seed's single batch generator is honoured)."""
        if kw.get("_noise") is not None:
            n = kw["_noise"]
            assert tuple(n.shape) == tuple(shape), (tuple(n.shape), shape)
            return n.to(device=self.device, dtype=self.dtype)
        return prepare_noise(shape, self.device, self.dtype, kw.get("seed"))

    def _use_steps(self) -> bool:
        """Schedule-wide timestep MLPs (acehip_dit_set_timesteps) for the bf16 runtime;
        ACEHIP_DIT_STEPS=0 runs every step through acehip_dit_forward (A/B)."""
        return (self.dtype == torch.bfloat16 and hasattr(self.rt, "set_timesteps")
                and os.environ.get("ACEHIP_DIT_STEPS", "1") != "0")

    def _set_cond(self, enc, cfg):
        if cfg:
            B = enc.shape[0]
            enc = torch.cat([enc, self.null.expand_as(enc)], dim=0)     # base:1907
            self.rt.set_condition(enc)
            # the null rows repeat one vector: closed-form cross-attention for them
            if self.uniform_null and self.null.numel() == enc.shape[-1]:
                self.rt.set_uniform_rows(B)
            return
        self.rt.set_condition(enc)

    def _base_loop(self, kw, enc, ctx, enc_nc, ctx_nc, acs):
        dtype, device = self.dtype, self.device
        B, T = ctx.shape[0], ctx.shape[1]
        infer_steps = int(kw.get("infer_steps", 30))
        guidance = float(kw.get("diffusion_guidance_sale", 7.0))
        shift = float(kw.get("shift", 1.0))
        method = kw.get("infer_method", "ode")
        use_adg = bool(kw.get("use_adg", False))
        t = base_schedule(infer_steps, shift, device, dtype,
                          kw.get("timesteps") if self.accepts_timesteps else None)
        noise = self._noise(kw, (B, T, ctx.shape[-1] // 2))
        cns = float(kw.get("cover_noise_strength", 0.0))
        if cns > 0.0:
            tv = t[:-1].tolist()
            nearest = min(tv, key=lambda x: abs(x - (1.0 - cns)))
            src = kw["src_latents"].to(device=device, dtype=dtype)
            xt = nearest * noise + (1 - nearest) * src          # renoise (base:1775-1781)
            t = t[tv.index(nearest):]
        else:
            xt = noise
        xt = xt.contiguous()
        n = len(t) - 1
        cover_steps = int(n * acs)
        do_cfg = guidance > 1.0
        # host copies of the schedule-derived scalars (one sync for the whole loop)
        dts = (t[:-1] - t[1:]).float().tolist()                        # bf16 t_curr − t_prev
        start, end = float(kw.get("cfg_interval_start", 0.0)), float(kw.get("cfg_interval_end", 1.0))
        cfg_on = ((t[:-1] >= start) & (t[:-1] <= end)).tolist()
        t_host = t.float().tolist()                                    # ADG sigma = t_curr
        t_dev = t.float().contiguous()
        self._set_cond(enc, do_cfg)
        ra = torch.zeros_like(xt) if do_cfg else None
        first = True
        switched = False
        steps_api = self._use_steps()
        if steps_api:
            self.rt.set_timesteps(t_dev[:n])
        for i in range(n):
            if i >= cover_steps and not switched:
                switched = True
                self._set_cond(enc_nc.to(device, dtype), do_cfg)
                ctx = ctx_nc.to(device=device, dtype=dtype).contiguous()
            vt = self.rt.forward_step(xt, ctx, i) if steps_api else self.rt.forward(xt, ctx, t_dev[i:i + 1])
            apply = (1 if cfg_on[i] else 0) if do_cfg else -1
            adg = use_adg and apply == 1          # ADG replaces APG inside the CFG interval (base:1949-1964)
            if method == "sde":
                if adg:
                    v = xt.clone()
                    adg_euler_(vt, v, guidance, t_host[i], 0.0, out_mode=1)
                else:
                    v = torch.empty_like(xt)
                    apg_euler_(vt, v, ra, guidance, 0.0, apply, first and apply == 1, out_mode=1)
                tc = t[i] * torch.ones((B,), device=device, dtype=dtype)
                x0 = xt - v * tc[:, None, None]
                nt = 1.0 - float(i + 1) / n
                xt = (nt * torch.randn_like(x0) + (1 - nt) * x0).contiguous()
            elif adg:
                adg_euler_(vt, xt, guidance, t_host[i], dts[i])
            else:
                apg_euler_(vt, xt, ra, guidance, dts[i], apply, first and apply == 1)
            if apply == 1:
                first = False
        return xt, n

    def _turbo_loop(self, kw, enc, ctx, enc_nc, ctx_nc, acs):
        dtype, device = self.dtype, self.device
        B, T = ctx.shape[0], ctx.shape[1]
        sched = turbo_schedule(float(kw.get("shift", 3.0)), kw.get("timesteps"))
        noise = self._noise(kw, (B, T, ctx.shape[-1] // 2))
        cns = float(kw.get("cover_noise_strength", 0.0))
        if cns > 0.0:
            nearest = min(sched, key=lambda x: abs(x - (1.0 - cns)))
            src = kw["src_latents"].to(device=device, dtype=dtype)
            xt = nearest * noise + (1 - nearest) * src
            sched = sched[sched.index(nearest):]
        else:
            xt = noise
        xt = xt.contiguous()
        tv = torch.tensor(sched, dtype=dtype).tolist()          # bf16-rounded table (.item())
        t_dev = torch.tensor(tv, dtype=torch.float32, device=device)
        n = len(tv)
        cover_steps = int(n * acs)
        method = kw.get("infer_method", "ode")
        self._set_cond(enc, False)
        switched = False
        steps_api = self._use_steps()
        if steps_api:
            self.rt.set_timesteps(t_dev[:n])
        for i in range(n):
            if i >= cover_steps and not switched:
                switched = True
                self._set_cond(enc_nc.to(device, dtype), False)
                ctx = ctx_nc.to(device=device, dtype=dtype).contiguous()
            vt = self.rt.forward_step(xt, ctx, i) if steps_api else self.rt.forward(xt, ctx, t_dev[i:i + 1])
            if i == n - 1:
                axpy_(vt, xt, tv[i])                               # x0 = xt − vt·t (turbo:1975-1977)
                break
            if method == "sde":
                tc = tv[i] * torch.ones((B,), device=device, dtype=dtype)
                x0 = xt - vt * tc[:, None, None]
                xt = (tv[i + 1] * torch.randn_like(x0) + (1 - tv[i + 1]) * x0).contiguous()
            else:
                dt = float((tv[i] - tv[i + 1]) * torch.ones(1, dtype=dtype))   # bf16(dt) (turbo:1988-1990)
                axpy_(vt, xt, dt)
        return xt, n
