"""Condition encoders on the HIP path: the ``AceStepConditionEncoder`` drop-in
and a ``prepare_condition`` drop-in built on it.

``ConditionEncoder.__call__`` keeps the contract of the reference
``AceStepConditionEncoder.forward`` (``acestep/models/base/
modeling_acestep_v15_base.py:1527-1554``): text projector, lyric encoder
(:577-731, key-padding masked), timbre encoder (:997-1178) and the two
``pack_sequences`` (:138-169) → ``(encoder_hidden_states, encoder_attention_mask)``.
Every Linear / encoder layer / norm runs in libacehip (``acehip_enc_*``,
``acehip_gemm_bf16``); the timbre unpack and ``pack_sequences`` are index
plumbing (stable argsort + gather) done with torch ops on the device, exactly
as the reference does them.  There is no CPU or eager fallback.

``AudioTokenizer`` / ``AudioDetokenizer`` are the cover
path's AceStepAudioTokenizer (attention pooler + FSQ) and AudioTokenDetokenizer
on the same encoder-stack runtime; the FSQ is a restatement of
``vector_quantize_pytorch`` (absent here: parity unpinned).

``HipPrepareCondition`` mirrors ``prepare_condition`` (base:1607-1652): the
encoders always, the tokenizer → detokenizer LM hints when a song is a cover
(with the tokenizer handles given; otherwise such songs go to the reference's
own ``prepare_condition`` when one is given, or raise).
"""
from __future__ import annotations

import logging
import math
from typing import Callable, Dict, Optional, Tuple

import torch

from . import _ffi
from ._ffi import ACEHIP_BF16, ACEHIP_F32, check, lib, ptr, shape_arg, stream_ptr
from .config import DiTConfig

log = logging.getLogger("acehip")


class EncoderStack:
    """One ``acehip_enc`` handle: embed_tokens → AceStepEncoderLayer × n →
    norm (→ proj_out), reference base:374-440."""

    def __init__(self, cfg: DiTConfig, n_layers: int, in_dim: int, embed_bias: bool = True,
                 out_dim: int = 0, device: int = 0, max_tokens: int = 8192, max_S: int = 4096,
                 causal: bool = False):
        self.cfg = cfg
        self.device = torch.device("cuda", device)
        self.D = cfg.hidden_size
        self.out_dim = out_dim
        self.max_tokens, self.max_S = max_tokens, max_S
        kinds = [2 if causal else (1 if cfg.is_sliding(i) else 0) for i in range(n_layers)]
        sl = (_ffi.c_uint8 * max(n_layers, 1))(*kinds)
        self._sliding = sl
        c = _ffi.EncCfg(hidden=cfg.hidden_size, intermediate=cfg.intermediate_size,
                        heads=cfg.num_attention_heads, kv_heads=cfg.num_key_value_heads,
                        head_dim=cfg.head_dim, layers=n_layers, window=cfg.sliding_window, in_dim=in_dim,
                        embed_bias=1 if embed_bias else 0, out_dim=out_dim, eps=cfg.rms_norm_eps,
                        rope_theta=cfg.rope_theta, max_tokens=max_tokens, max_S=max_S,
                        sliding=_ffi.ctypes.cast(sl, _ffi.POINTER(_ffi.c_uint8)))
        h = _ffi.c_void_p()
        check(lib().acehip_enc_create(device, _ffi.ctypes.byref(c), _ffi.ctypes.byref(h)), "enc_create")
        self.h = h
        self.extra: Dict[str, torch.Tensor] = {}   # special_token(s): host-side plumbing parameters

    def set_weight(self, name: str, t: torch.Tensor):
        t = t.detach().contiguous()
        if t.dtype not in (torch.float32, torch.bfloat16):
            t = t.float()
        dt = ACEHIP_F32 if t.dtype == torch.float32 else ACEHIP_BF16
        check(lib().acehip_enc_set_weight(self.h, name.encode(), ptr(t), dt, t.dim(), shape_arg(tuple(t.shape)),
                                          1 if t.is_cuda else 0), f"enc_set_weight({name})")

    def load(self, weights: Dict[str, torch.Tensor], prefix: str = ""):
        """Module-local reference names under ``prefix`` (e.g. ``lyric_encoder.``)."""
        hd = self.cfg.head_dim
        inv = 1.0 / (self.cfg.rope_theta ** (torch.arange(0, hd, 2, dtype=torch.float) / hd))
        self.set_weight("_rope_inv_freq", inv)
        for k, v in weights.items():
            if not k.startswith(prefix):
                continue
            k = k[len(prefix):]
            if k.startswith("rotary_emb."):
                continue
            if k in ("special_token", "special_tokens"):
                self.extra[k] = v.detach().to(self.device, torch.bfloat16)
                continue
            self.set_weight(k, v)
        check(lib().acehip_enc_finalize(self.h), "enc_finalize")

    def embed(self, x: torch.Tensor) -> torch.Tensor:
        x = x.to(self.device, torch.bfloat16).contiguous()
        M = x.numel() // x.shape[-1]
        out = torch.empty(*x.shape[:-1], self.D, device=self.device, dtype=torch.bfloat16)
        check(lib().acehip_enc_embed(self.h, ptr(x), M, ptr(out), stream_ptr()), "enc_embed")
        return out

    def forward(self, h: torch.Tensor, kmask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """h [B, S, D] bf16 (embedded) → [B, S, out_dim or D]; kmask [B, S] (1 = attend) or None."""
        h = h.to(self.device, torch.bfloat16).contiguous()
        B, S, _ = h.shape
        km = None
        if kmask is not None:
            km = (kmask != 0).to(device=self.device, dtype=torch.uint8).contiguous()
        out = torch.empty(B, S, self.out_dim or self.D, device=self.device, dtype=torch.bfloat16)
        check(lib().acehip_enc_forward(self.h, ptr(h), ptr(km), B, S, ptr(out), stream_ptr()), "enc_forward")
        self._keep = (h, km)   # inputs stay alive until the stream consumed them
        return out

    def close(self):
        if getattr(self, "h", None):
            lib().acehip_enc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _EmbedTokens:
    """``text_encoder.embed_tokens(ids)``: the embedding-table row gather (index plumbing
    on the device, as the reference's nn.Embedding does it)."""

    def __init__(self, table: torch.Tensor):
        self.weight = table

    def __call__(self, input_ids: torch.Tensor) -> torch.Tensor:
        return torch.nn.functional.embedding(input_ids.to(self.weight.device), self.weight)


class TextEncoderOutput:
    def __init__(self, last_hidden_state: torch.Tensor):
        self.last_hidden_state = last_hidden_state


def await_ready(t: Optional[torch.Tensor]) -> None:
    """Make the current stream wait for a tensor that an overlapped ``TextEncoder`` is still
    producing on its side stream (``_acehip_ready``, set by ``TextEncoder(overlap=True)``)."""
    ev = getattr(t, "_acehip_ready", None)
    if ev is not None:
        torch.cuda.current_stream(t.device).wait_event(ev)


class TextEncoder:
    """Qwen3-Embedding-0.6B (``Qwen3Model``) drop-in for the reference's ``text_encoder``
    (loaded at ``init_service_loader.py:146-160``, called by ``infer_text_embeddings`` /
    ``infer_lyric_embeddings``, ``conditioning_embed.py:71-79``):
    ``text_encoder(input_ids=ids, lyric_attention_mask=None).last_hidden_state`` and
    ``text_encoder.embed_tokens(ids)``.  The 28 causal Qwen3 decoder layers and the final
    norm run on the ``acehip_enc`` runtime (every layer causal, no embed Linear); the
    embedding lookup is a device gather.  Like the reference call (no ``attention_mask``)
    the mask is Qwen3Model's default causal one; a padding mask is not supported."""

    QWEN3_06B = dict(hidden_size=1024, intermediate_size=3072, num_hidden_layers=28, num_attention_heads=16,
                     num_key_value_heads=8, head_dim=128, rms_norm_eps=1e-6, rope_theta=1_000_000.0)

    def __init__(self, cfg: Optional[DiTConfig] = None, device: int = 0, max_batch: int = 8, max_tokens: int = 512,
                 overlap: bool = False):
        self.cfg = cfg or DiTConfig(**self.QWEN3_06B)
        self.device = torch.device("cuda", device)
        self.stack = EncoderStack(self.cfg, self.cfg.num_hidden_layers, 0, device=device,
                                  max_tokens=max_batch * max_tokens, max_S=max_tokens, causal=True)
        self.embed_tokens: Optional[_EmbedTokens] = None
        # overlap=True: the 28 layers run on a side stream and the call returns at once; the
        # output carries the side stream's completion event (``_acehip_ready``), which the
        # condition encoder waits for only after its lyric and timbre encoders are queued, so
        # the independent encoder chains overlap.  Opt-in: a consumer that is not acehip's
        # must call ``await_ready(last_hidden_state)`` before touching the tensor.
        self._side = torch.cuda.Stream(self.device) if overlap else None

    @classmethod
    def from_reference_model(cls, model, **kw) -> "TextEncoder":
        """From the reference's loaded ``AutoModel`` (a transformers ``Qwen3Model``)."""
        c = model.config
        cfg = DiTConfig(hidden_size=c.hidden_size, intermediate_size=c.intermediate_size,
                        num_hidden_layers=c.num_hidden_layers, num_attention_heads=c.num_attention_heads,
                        num_key_value_heads=c.num_key_value_heads,
                        head_dim=getattr(c, "head_dim", c.hidden_size // c.num_attention_heads),
                        rms_norm_eps=c.rms_norm_eps, rope_theta=_rope_theta(c))
        te = cls(cfg, **kw)
        te.load(model.state_dict())
        return te

    def load(self, weights: Dict[str, torch.Tensor]):
        """Qwen3Model state-dict names (``embed_tokens.weight``, ``layers.N.…``, ``norm.weight``)."""
        w = {k: v for k, v in weights.items() if k != "embed_tokens.weight"}
        self.embed_tokens = _EmbedTokens(weights["embed_tokens.weight"].detach().to(self.device, torch.bfloat16))
        self.stack.load(w)

    def __call__(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                 **kwargs) -> TextEncoderOutput:
        if attention_mask is not None:
            raise NotImplementedError("TextEncoder: padding masks are not supported (the reference passes none)")
        if self._side is None:
            h = self.embed_tokens(input_ids)
            return TextEncoderOutput(self.stack.forward(h))
        main = torch.cuda.current_stream(self.device)
        self._side.wait_stream(main)                 # input ids (and the weights) ready
        with torch.cuda.stream(self._side):
            h = self.embed_tokens(input_ids)
            out = self.stack.forward(h)
        ev = torch.cuda.Event()
        ev.record(self._side)
        out.record_stream(main)                      # read on the consumer's stream later
        out._acehip_ready = ev
        return TextEncoderOutput(out)

    def to(self, *a, **k) -> "TextEncoder":
        """The handler's offload context moves models with ``.to``; the handle stays resident."""
        return self

    def eval(self) -> "TextEncoder":
        return self

    def close(self):
        self.stack.close()


def _rope_theta(c) -> float:
    rp = getattr(c, "rope_parameters", None) or {}
    return float(rp.get("rope_theta", getattr(c, "rope_theta", 1_000_000.0)))


def timbre_layout(order: torch.Tensor) -> Tuple[int, int]:
    """(batch size, max references per song) of a packed-timbre order vector (host values)."""
    o = order.long().flatten().tolist()
    B = max(o) + 1
    return B, max(o.count(b) for b in range(B))


def unpack_timbre(emb: torch.Tensor, order: torch.Tensor,
                  layout: Optional[Tuple[int, int]] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """AceStepTimbreEncoder.unpack_timbre_embeddings (base:1023-1073): packed rows
    [N, d] → [B, max_count, d] by batch id in packed order, mask [B, max_count] long.
    (The reference's one-hot matmul places each row exactly; an index scatter
    is the same result.)  `layout` = timbre_layout(order) when already known (no host sync)."""
    N, d = emb.shape
    dev = emb.device
    order = order.to(dev).long()
    B, max_count = layout if layout is not None else timbre_layout(order)
    counts = torch.bincount(order, minlength=B)
    sorted_idx = torch.argsort(order * N + torch.arange(N, device=dev), stable=True)
    starts = torch.cat([torch.zeros(1, dtype=torch.long, device=dev), torch.cumsum(counts, 0)[:-1]])
    pos_sorted = torch.arange(N, device=dev) - starts[order[sorted_idx]]
    pos = torch.empty_like(pos_sorted)
    pos[sorted_idx] = pos_sorted
    out = torch.zeros(B * max_count, d, device=dev, dtype=emb.dtype)
    out[order * max_count + pos] = emb
    mask = torch.zeros(B * max_count, dtype=torch.long, device=dev)
    mask[order * max_count + pos] = 1
    return out.view(B, max_count, d), mask.view(B, max_count)


def pack_sequences(h1, h2, m1, m2):
    """pack_sequences (base:138-169): valid tokens first (stable), prefix mask."""
    h = torch.cat([h1, h2], dim=1)
    m = torch.cat([m1.to(h.device), m2.to(h.device)], dim=1)
    B, L, D = h.shape
    idx = m.argsort(dim=1, descending=True, stable=True)
    out = torch.gather(h, 1, idx.unsqueeze(-1).expand(B, L, D))
    lengths = m.sum(dim=1)
    return out, torch.arange(L, device=h.device)[None, :] < lengths[:, None]


class ConditionEncoder:
    """Drop-in for ``AceStepConditionEncoder`` (base:1509-1554) on libacehip."""

    def __init__(self, cfg: DiTConfig, device: int = 0, max_batch: int = 8, max_lyric: int = 4096,
                 max_refs: int = 8, max_ref_frames: int = 750):
        self.cfg = cfg
        self.device = torch.device("cuda", device)
        self.lyric = EncoderStack(cfg, cfg.num_lyric_encoder_hidden_layers, cfg.text_hidden_dim, True,
                                  device=device, max_tokens=max_batch * max_lyric, max_S=max_lyric)
        self.timbre = EncoderStack(cfg, cfg.num_timbre_encoder_hidden_layers, cfg.timbre_hidden_dim, True,
                                   device=device, max_tokens=max_refs * max_ref_frames, max_S=max_ref_frames)
        self.w_text: Optional[torch.Tensor] = None

    @classmethod
    def from_reference_model(cls, model, **kw) -> "ConditionEncoder":
        """From a loaded ``AceStepConditionGenerationModel`` (its ``encoder`` submodule)."""
        c = model.config
        cfg = DiTConfig(hidden_size=c.hidden_size, intermediate_size=c.intermediate_size,
                        num_hidden_layers=c.num_hidden_layers, num_attention_heads=c.num_attention_heads,
                        num_key_value_heads=c.num_key_value_heads, head_dim=c.head_dim,
                        sliding_window=c.sliding_window, rms_norm_eps=c.rms_norm_eps,
                        rope_theta=float(getattr(c, "rope_theta", 1e6)), layer_types=list(c.layer_types),
                        num_lyric_encoder_hidden_layers=c.num_lyric_encoder_hidden_layers,
                        num_timbre_encoder_hidden_layers=c.num_timbre_encoder_hidden_layers,
                        num_attention_pooler_hidden_layers=c.num_attention_pooler_hidden_layers,
                        pool_window_size=c.pool_window_size, audio_acoustic_hidden_dim=c.audio_acoustic_hidden_dim,
                        text_hidden_dim=c.text_hidden_dim, timbre_hidden_dim=c.timbre_hidden_dim)
        dev = next(model.parameters()).device
        ce = cls(cfg, dev.index or 0, **kw)
        ce.load(model.encoder.state_dict())
        return ce

    def load(self, weights: Dict[str, torch.Tensor]):
        w = {(k[len("encoder."):] if k.startswith("encoder.") else k): v for k, v in weights.items()}
        self.w_text = w["text_projector.weight"].detach().to(self.device, torch.bfloat16).contiguous()
        self.lyric.load(w, "lyric_encoder.")
        self.timbre.load(w, "timbre_encoder.")

    def text_projector(self, text: torch.Tensor) -> torch.Tensor:
        """nn.Linear(text_hidden_dim → hidden, bias=False) (base:1521, :1540)."""
        x = text.to(self.device, torch.bfloat16).contiguous()
        M, K = x.numel() // x.shape[-1], x.shape[-1]
        N = self.w_text.shape[0]
        out = torch.empty(*x.shape[:-1], N, device=self.device, dtype=torch.bfloat16)
        check(lib().acehip_gemm_bf16(ptr(x), K, ptr(self.w_text), K, ptr(out), N, M, N, K, None, stream_ptr()),
              "text_projector")
        return out

    def lyric_encoder(self, lyric_hidden_states, lyric_attention_mask):
        """AceStepLyricEncoder.forward (base:603-731) → last_hidden_state."""
        return self.lyric.forward(self.lyric.embed(lyric_hidden_states), lyric_attention_mask)

    def timbre_encoder(self, packed, order, layout=None):
        """AceStepTimbreEncoder.forward (base:1076-1178): no padding mask, row 0."""
        h = self.timbre.forward(self.timbre.embed(packed), None)
        return unpack_timbre(h[:, 0, :], order, layout)

    def __call__(self, text_hidden_states, text_attention_mask, lyric_hidden_states, lyric_attention_mask,
                 refer_audio_acoustic_hidden_states_packed, refer_audio_order_mask):
        dev = self.device
        # lyric and timbre first: an overlapped text encoder (TextEncoder(overlap=True)) is
        # waited for only after them (the three chains are independent; results unchanged)
        lyric = self.lyric_encoder(lyric_hidden_states, lyric_attention_mask)
        timbre, timbre_mask = self.timbre_encoder(refer_audio_acoustic_hidden_states_packed, refer_audio_order_mask)
        await_ready(text_hidden_states)
        text = self.text_projector(text_hidden_states)
        enc, mask = pack_sequences(lyric, timbre, lyric_attention_mask.to(dev), timbre_mask)
        return pack_sequences(enc, text, mask, text_attention_mask.to(dev))

    forward = __call__

    def close(self):
        self.lyric.close()
        self.timbre.close()


FSQ_LEVELS = (8, 8, 8, 5, 5, 5)      # configuration_acestep_v15.py:152


def _gemm(x: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor]) -> torch.Tensor:
    """bf16 x [.., K] · Wᵀ (+ b) on libacehip (N % 128, K % 64)."""
    x = x.contiguous()
    M, K = x.numel() // x.shape[-1], x.shape[-1]
    N = W.shape[0]
    out = torch.empty(*x.shape[:-1], N, device=x.device, dtype=torch.bfloat16)
    check(lib().acehip_gemm_bf16(ptr(x), K, ptr(W), K, ptr(out), N, M, N, K, ptr(b), stream_ptr()), "gemm")
    return out


def _pad_rows(w: torch.Tensor, rows: int, dev) -> torch.Tensor:
    out = torch.zeros(rows, *w.shape[1:], device=dev, dtype=torch.bfloat16)
    out[: w.shape[0]] = w.detach().to(dev, torch.bfloat16)
    return out.contiguous()


class AudioTokenizer:
    """AceStepAudioTokenizer (base:1181-1223) on libacehip: audio_acoustic_proj →
    AttentionPooler (base:734-859: embed, special token first, encoder layers on
    (P+1)-token sequences, norm, CLS) → ResidualFSQ (project_in → FSQ → project_out;
    the FSQ restated from vector_quantize_pytorch's published algorithm — the
    library is not in this image, so its parity is unpinned)."""

    def __init__(self, cfg: DiTConfig, device: int = 0, max_patches: int = 3000):
        self.cfg, self.P = cfg, cfg.pool_window_size
        self.device = torch.device("cuda", device)
        self.pooler = EncoderStack(cfg, cfg.num_attention_pooler_hidden_layers, cfg.hidden_size, True,
                                   device=device, max_tokens=max_patches * (self.P + 1), max_S=self.P + 1)
        self._levels = (_ffi.c_int * len(FSQ_LEVELS))(*FSQ_LEVELS)

    def load(self, weights: Dict[str, torch.Tensor], prefix: str = "tokenizer."):
        w = {k[len(prefix):]: v for k, v in weights.items() if k.startswith(prefix)}
        dev = self.device
        self.w_proj = w["audio_acoustic_proj.weight"].detach().to(dev, torch.bfloat16).contiguous()
        self.b_proj = w["audio_acoustic_proj.bias"].detach().to(dev, torch.bfloat16).contiguous()
        self.pooler.load(w, "attention_pooler.")
        nl = len(FSQ_LEVELS)
        # project_in [6, D] rows padded to 128; project_out [D, 6] columns padded to 64 (K)
        self.w_in = _pad_rows(w["quantizer.project_in.weight"], 128, dev)
        self.b_in = _pad_rows(w["quantizer.project_in.bias"], 128, dev)
        wo = torch.zeros(w["quantizer.project_out.weight"].shape[0], 64, device=dev, dtype=torch.bfloat16)
        wo[:, :nl] = w["quantizer.project_out.weight"].detach().to(dev, torch.bfloat16)
        self.w_out = wo.contiguous()
        self.b_out = w["quantizer.project_out.bias"].detach().to(dev, torch.bfloat16).contiguous()

    def project_out(self, codes64: torch.Tensor) -> torch.Tensor:
        return _gemm(codes64, self.w_out, self.b_out)

    def quantize(self, h: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """ResidualFSQ.forward (1 quantizer): h [.., D] → (quantized [.., D], indices [.., 1] int32)."""
        z = _gemm(h, self.w_in, self.b_in)                        # [.., 128], first 6 columns real
        M = z.numel() // 128
        codes = torch.empty(M, 64, device=self.device, dtype=torch.bfloat16)
        idx = torch.empty(M, device=self.device, dtype=torch.int32)
        check(lib().acehip_fsq_quantize(ptr(z), 128, M, self._levels, len(FSQ_LEVELS), ptr(codes), 64, ptr(idx),
                                        stream_ptr()), "fsq_quantize")
        q = self.project_out(codes).view(*h.shape[:-1], -1)
        return q, idx.view(*h.shape[:-1], 1)

    def get_output_from_indices(self, indices: torch.Tensor) -> torch.Tensor:
        """ResidualFSQ.get_output_from_indices (used by audio_codes.py:62): [.., 1] → [.., D]."""
        idx = indices.to(self.device, torch.int32).contiguous()
        M = idx.numel()
        codes = torch.empty(M, 64, device=self.device, dtype=torch.bfloat16)
        check(lib().acehip_fsq_codes_from_indices(ptr(idx), M, self._levels, len(FSQ_LEVELS), ptr(codes), 64,
                                                  stream_ptr()), "fsq_codes")
        return self.project_out(codes).view(*indices.shape[:-1], -1)

    def attention_pooler(self, x: torch.Tensor) -> torch.Tensor:
        """x [N, T, P, D] (embedded by audio_acoustic_proj) → CLS [N, T, D]."""
        N, T, P, D = x.shape
        h = self.pooler.embed(x)
        sp = self.pooler.extra["special_token"].expand(N, T, 1, D)
        h = torch.cat([sp, h], dim=2).reshape(N * T, P + 1, D)
        return self.pooler.forward(h, None)[:, 0, :].reshape(N, T, D)

    def __call__(self, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """AceStepAudioTokenizer.forward: x [N, T/P, P, 64] → (quantized, indices)."""
        h = _gemm(x.to(self.device, torch.bfloat16), self.w_proj, self.b_proj)
        return self.quantize(self.attention_pooler(h))

    def close(self):
        self.pooler.close()


class AudioDetokenizer:
    """AudioTokenDetokenizer (base:862-994) on libacehip: embed, repeat each token
    P times + the learned special tokens (a bf16 add, as the reference), encoder
    layers on P-token sequences, norm, proj_out → 25 Hz latents."""

    def __init__(self, cfg: DiTConfig, device: int = 0, max_patches: int = 3000):
        self.cfg, self.P = cfg, cfg.pool_window_size
        self.stack = EncoderStack(cfg, cfg.num_attention_pooler_hidden_layers, cfg.hidden_size, True,
                                  out_dim=cfg.audio_acoustic_hidden_dim, device=device,
                                  max_tokens=max_patches * self.P, max_S=self.P)

    def load(self, weights: Dict[str, torch.Tensor], prefix: str = "detokenizer."):
        self.stack.load(weights, prefix)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        N, T, D = x.shape
        h = self.stack.embed(x)
        h = h.unsqueeze(2).repeat(1, 1, self.P, 1) + self.stack.extra["special_tokens"].expand(N, T, -1, -1)
        out = self.stack.forward(h.reshape(N * T, self.P, D), None)
        return out.reshape(N, T * self.P, -1)

    def close(self):
        self.stack.close()


class HipPrepareCondition:
    """Drop-in for ``AceStepConditionGenerationModel.prepare_condition``
    (base:1607-1652) with the encoders on libacehip.

    The reference always runs the audio tokenizer/detokenizer and then keeps
    its output only where ``is_covers > 0`` (base:1645-1649); without covers
    (or with ``precomputed_lm_hints_25Hz``) that work is dead and skipped here.
    Covers that need the tokenizer go to ``fallback`` (the reference's own
    ``prepare_condition``) or raise."""

    # the inputs the result depends on (``attention_mask`` only feeds tokenize's pooled mask,
    # which prepare_condition discards: base:1586-1590,1645)
    _MEMO_KEYS = ("text_hidden_states", "text_attention_mask", "lyric_hidden_states", "lyric_attention_mask",
                  "refer_audio_acoustic_hidden_states_packed", "refer_audio_order_mask", "hidden_states",
                  "silence_latent", "src_latents", "chunk_masks", "is_covers", "precomputed_lm_hints_25Hz",
                  "audio_codes")

    def __init__(self, encoder: ConditionEncoder, fallback: Optional[Callable] = None,
                 tokenizer: Optional[AudioTokenizer] = None, detokenizer: Optional[AudioDetokenizer] = None):
        self.encoder = encoder
        self.fallback = fallback
        self.tokenizer, self.detokenizer = tokenizer, detokenizer
        self._memo = None
        self.passes = 0          # encoder passes run (tests count one per request through install())

    # -- one encoder pass per request ------------------------------------------------------------
    # The handler conditions the request itself (service_generate_execute.py:123-142) and the
    # reference generate_audio conditions it AGAIN from the same payload tensors (base:1820).
    # install() binds ``record`` to the handler's call and ``consume`` to generate_audio's: the
    # second call reuses the first's outputs when every input is the same tensor object (same
    # storage, shape and — where torch tracks one — version); the memo is single-use, so a later
    # request (or a direct generate_audio call, as bench.py makes) always runs the encoders.
    @classmethod
    def _key(cls, kw):
        parts = []
        for name in cls._MEMO_KEYS:
            v = kw.get(name)
            if isinstance(v, torch.Tensor):
                try:
                    ver = v._version
                except RuntimeError:             # inference tensors carry no version counter
                    ver = None
                parts.append((name, id(v), v.data_ptr(), tuple(v.shape), v.dtype, ver))
            else:
                parts.append((name, None if v is None else ("obj", id(v))))
        return tuple(parts)

    def record(self, **kw):
        out = self(**kw)
        # strong references keep the keyed objects (and so their ids) alive while the memo lives
        self._memo = (self._key(kw), [kw.get(n) for n in self._MEMO_KEYS], out)
        return out

    def consume(self, **kw):
        memo, self._memo = self._memo, None
        if memo is not None and memo[0] == self._key(kw):
            return memo[2]
        return self(**kw)

    def tokenize(self, x, silence_latent):
        """AceStepConditionGenerationModel.tokenize (base:1580-1591): pad T to a
        multiple of P with the silence latent, group P frames, tokenize."""
        P = self.tokenizer.P
        if x.shape[1] % P:
            pad = P - x.shape[1] % P
            x = torch.cat([x, silence_latent[:1, :pad].to(x.dtype).repeat(x.shape[0], 1, 1)], dim=1)
        return self.tokenizer(x.reshape(x.shape[0], -1, P, x.shape[-1]))

    def __call__(self, text_hidden_states, text_attention_mask, lyric_hidden_states, lyric_attention_mask,
                 refer_audio_acoustic_hidden_states_packed, refer_audio_order_mask, hidden_states,
                 attention_mask, silence_latent, src_latents, chunk_masks, is_covers,
                 precomputed_lm_hints_25Hz=None, audio_codes=None):
        need_tokenizer = precomputed_lm_hints_25Hz is None and (
            audio_codes is not None or bool((is_covers > 0).any()))
        if need_tokenizer and self.tokenizer is not None and self.detokenizer is not None:
            # base:1641-1649: LM hints from the source latents (or from audio codes)
            if audio_codes is not None:
                q = self.tokenizer.get_output_from_indices(audio_codes)
            else:
                q, _ = self.tokenize(hidden_states.to(torch.bfloat16), silence_latent)
            precomputed_lm_hints_25Hz = self.detokenizer(q).to(hidden_states.dtype)
            need_tokenizer = False
        if need_tokenizer:
            await_ready(text_hidden_states)          # the reference's code reads it at once
            if self.fallback is None:
                raise NotImplementedError("acehip: cover conditioning needs the FSQ audio tokenizer "
                                          "(pass precomputed_lm_hints_25Hz or a reference fallback)")
            log.warning("acehip: cover conditioning without an audio tokenizer handle — delegating this "
                        "request to the reference prepare_condition (PyTorch, not libacehip)")
            return self.fallback(
                text_hidden_states=text_hidden_states, text_attention_mask=text_attention_mask,
                lyric_hidden_states=lyric_hidden_states, lyric_attention_mask=lyric_attention_mask,
                refer_audio_acoustic_hidden_states_packed=refer_audio_acoustic_hidden_states_packed,
                refer_audio_order_mask=refer_audio_order_mask, hidden_states=hidden_states,
                attention_mask=attention_mask, silence_latent=silence_latent, src_latents=src_latents,
                chunk_masks=chunk_masks, is_covers=is_covers,
                precomputed_lm_hints_25Hz=precomputed_lm_hints_25Hz, audio_codes=audio_codes)
        dtype = hidden_states.dtype
        self.passes += 1
        enc, enc_mask = self.encoder(text_hidden_states, text_attention_mask, lyric_hidden_states,
                                     lyric_attention_mask, refer_audio_acoustic_hidden_states_packed,
                                     refer_audio_order_mask)
        if precomputed_lm_hints_25Hz is not None:
            hints = precomputed_lm_hints_25Hz[:, :src_latents.shape[1], :]
            src_latents = torch.where(is_covers.view(-1, 1, 1) > 0, hints, src_latents)
        ctx = torch.cat([src_latents, chunk_masks.to(dtype)], dim=-1)
        return enc.to(dtype), enc_mask, ctx
