"""ctypes binding of libacehip.so (C ABI declared in include/acehip.h).

The library is built in-tree (``make -C ace-step-1.5_amd`` or
``__graft_entry__.build()``) and loaded from this directory.  There is no
fallback: if the shared object is missing or fails to load, every entry point
raises — the product path never silently degrades to a CPU/eager path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_int64, c_uint8, c_void_p

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libacehip.so")

ACEHIP_F32 = 0
ACEHIP_BF16 = 1
# include/acehip.h ACEHIP_VERSION this binding's signatures were written against
ABI_VERSION = 400

# every symbol include/acehip.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "acehip_get_version", "acehip_last_error", "acehip_reload_knobs", "acehip_build_hash",
    "acehip_dit_create", "acehip_dit_set_weight", "acehip_dit_finalize",
    "acehip_dit_set_condition", "acehip_dit_set_uniform_rows", "acehip_dit_forward", "acehip_dit_destroy",
    "acehip_dit_set_graph", "acehip_dit_set_timesteps", "acehip_dit_forward_step",
    "acehip_dit_profile", "acehip_dit_profile_read", "acehip_dit_profile_kinds",
    "acehip_sampler_apg_euler", "acehip_sampler_adg_euler", "acehip_sampler_axpy",
    "acehip_vae_create", "acehip_vae_set_weight", "acehip_vae_finalize", "acehip_vae_decode",
    "acehip_vae_decode_blocks",
    "acehip_vae_encode", "acehip_vae_destroy", "acehip_vae_conv", "acehip_vae_resunit",
    "acehip_wav_peak_normalize", "acehip_wav_postprocess", "acehip_wav_postprocess_pcm16",
    "acehip_gemm_bf16", "acehip_gemm_bf16_ex", "acehip_attention_bf16",
    "acehip_rmsnorm_bf16", "acehip_gemm_headpost_bf16", "acehip_attention_masked_bf16",
    "acehip_enc_create", "acehip_enc_set_weight", "acehip_enc_finalize", "acehip_enc_embed",
    "acehip_enc_forward", "acehip_enc_destroy", "acehip_fsq_quantize", "acehip_fsq_codes_from_indices",
]


class DiTCfg(ctypes.Structure):
    _fields_ = [("hidden", c_int), ("intermediate", c_int), ("heads", c_int), ("kv_heads", c_int),
                ("head_dim", c_int), ("layers", c_int), ("window", c_int), ("patch", c_int),
                ("in_channels", c_int), ("out_channels", c_int), ("eps", c_float),
                ("rope_theta", c_float), ("max_S", c_int), ("max_Bc", c_int), ("max_Lenc", c_int),
                ("sliding", POINTER(c_uint8)), ("fp32", c_int)]


class EncCfg(ctypes.Structure):
    _fields_ = [("hidden", c_int), ("intermediate", c_int), ("heads", c_int), ("kv_heads", c_int),
                ("head_dim", c_int), ("layers", c_int), ("window", c_int), ("in_dim", c_int),
                ("embed_bias", c_int), ("out_dim", c_int), ("eps", c_float), ("rope_theta", c_float),
                ("max_tokens", c_int), ("max_S", c_int), ("sliding", POINTER(c_uint8))]


class VAECfg(ctypes.Structure):
    _fields_ = [("encoder_hidden", c_int), ("decoder_channels", c_int), ("latent_channels", c_int),
                ("audio_channels", c_int), ("n_blocks", c_int), ("ratios", c_int * 8),
                ("multiples", c_int * 8), ("max_T", c_int), ("max_B", c_int),
                ("with_encoder", c_int)]


_LIB = None


def _declare(lib):
    P = c_void_p
    sig = {
        "acehip_get_version": (c_int, []),
        "acehip_last_error": (c_char_p, []),
        "acehip_build_hash": (c_char_p, []),
        "acehip_reload_knobs": (c_int, []),
        "acehip_dit_create": (c_int, [c_int, POINTER(DiTCfg), POINTER(c_void_p)]),
        "acehip_dit_set_weight": (c_int, [P, c_char_p, P, c_int, c_int, POINTER(c_int64), c_int]),
        "acehip_dit_finalize": (c_int, [P]),
        "acehip_dit_set_condition": (c_int, [P, P, c_int, c_int, P]),
        "acehip_dit_set_uniform_rows": (c_int, [P, c_int, P]),
        "acehip_dit_forward": (c_int, [P, P, P, c_int, P, P, c_int, c_int, c_int, c_int, P, P]),
        "acehip_dit_destroy": (c_int, [P]),
        "acehip_dit_set_graph": (c_int, [P, c_int]),
        "acehip_dit_set_timesteps": (c_int, [P, P, P, c_int, P]),
        "acehip_dit_forward_step": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, P, P]),
        "acehip_dit_profile": (c_int, [P, c_int]),
        "acehip_dit_profile_kinds": (c_int, [P, ctypes.c_uint]),
        "acehip_dit_profile_read": (c_int, [P, c_int, POINTER(c_int), POINTER(c_float)]),
        "acehip_sampler_apg_euler": (c_int, [P, P, P, c_int, c_int, c_int, c_float, c_float, c_int,
                                             c_int, c_int, c_int, P]),
        "acehip_sampler_adg_euler": (c_int, [P, P, c_int, c_int, c_int, c_float, c_float, c_float, c_int, c_int, P]),
        "acehip_sampler_axpy": (c_int, [P, P, c_int64, c_float, c_int, P]),
        "acehip_vae_create": (c_int, [c_int, POINTER(VAECfg), POINTER(c_void_p)]),
        "acehip_vae_set_weight": (c_int, [P, c_char_p, P, c_int, c_int, POINTER(c_int64), c_int]),
        "acehip_vae_finalize": (c_int, [P]),
        "acehip_vae_decode": (c_int, [P, P, c_int, c_int, P, P]),
        "acehip_vae_decode_blocks": (c_int, [P, P, c_int, c_int, P, P]),
        "acehip_vae_encode": (c_int, [P, P, c_int, c_int, P, P, P]),
        "acehip_vae_destroy": (c_int, [P]),
        "acehip_vae_conv": (c_int, [c_int, P, c_int64, c_int, P, P, P, c_int, c_int, c_int, c_int, P, P, P, P, P]),
        "acehip_vae_resunit": (c_int, [P, P, c_int64, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P]),
        "acehip_wav_peak_normalize": (c_int, [P, c_int, c_int64, P, P]),
        "acehip_wav_postprocess": (c_int, [P, c_int, c_int64, P, c_int, c_float, P]),
        "acehip_wav_postprocess_pcm16": (c_int, [P, c_int, c_int, c_int64, P, c_int, c_float, P, P]),
        "acehip_gemm_bf16": (c_int, [P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, P, P]),
        "acehip_gemm_bf16_ex": (c_int, [P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, P, c_int,
                                        c_int, P]),
        "acehip_attention_bf16": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int,
                                          c_float, P]),
        "acehip_attention_masked_bf16": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int,
                                                 c_float, P, P]),
        "acehip_enc_create": (c_int, [c_int, POINTER(EncCfg), POINTER(c_void_p)]),
        "acehip_enc_set_weight": (c_int, [P, c_char_p, P, c_int, c_int, POINTER(c_int64), c_int]),
        "acehip_enc_finalize": (c_int, [P]),
        "acehip_enc_embed": (c_int, [P, P, c_int, P, P]),
        "acehip_enc_forward": (c_int, [P, P, P, c_int, c_int, P, P]),
        "acehip_enc_destroy": (c_int, [P]),
        "acehip_fsq_quantize": (c_int, [P, c_int, c_int, POINTER(c_int), c_int, P, c_int, P, P]),
        "acehip_fsq_codes_from_indices": (c_int, [P, c_int, POINTER(c_int), c_int, P, c_int, P]),
        "acehip_rmsnorm_bf16": (c_int, [P, P, P, P, c_int64, c_int, P, c_int, c_int, c_float, c_int, P]),
        "acehip_gemm_headpost_bf16": (c_int, [P, c_int, P, c_int, c_int, c_int, c_int, c_int, c_int,
                                              P, P, P, P, c_float, P, P, P, P]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(lib, name):
            continue  # reported by missing_exports()
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib():
    """Load libacehip.so (raises if it is missing — no fallback path exists)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"acehip: {LIB_PATH} not built; run `make -C ace-step-1.5_amd` "
                               "or __graft_entry__.build()")
        handle = ctypes.CDLL(LIB_PATH)
        _declare(handle)
        v = handle.acehip_get_version()
        if v != ABI_VERSION:
            raise RuntimeError(f"acehip: {LIB_PATH} has ABI version {v}, this binding expects "
                               f"{ABI_VERSION} (include/acehip.h); rebuild the library")
        built, tree = build_hash(handle), source_hash()
        if tree is not None and built != tree:
            raise RuntimeError(f"acehip: {LIB_PATH} was built from native sources {built}, the tree beside "
                               f"it is {tree}; rebuild the library (make -C ace-step-1.5_amd)")
        _LIB = handle
    return _LIB


def build_hash(handle=None) -> str:
    """The native-source hash compiled into the library (acehip_build_hash)."""
    h = handle if handle is not None else lib()
    if not hasattr(h, "acehip_build_hash"):
        return "none"
    h.acehip_build_hash.restype = c_char_p
    return h.acehip_build_hash().decode()


def source_hash():
    """The native-source hash of the tree this package sits in (None if the sources are absent,
    e.g. an installed wheel: then only the ABI version is checked)."""
    script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "native_hash.py")
    if not os.path.exists(script):
        return None
    import importlib.util
    spec = importlib.util.spec_from_file_location("_acehip_native_hash", script)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.native_hash()


def missing_exports():
    l = lib()
    return [n for n in EXPORTS if not hasattr(l, n)]


def reload_knobs():
    """Re-read the ACEHIP_* A/B switches after changing the environment (tests / A/B tools)."""
    check(lib().acehip_reload_knobs(), "reload_knobs")


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().acehip_last_error()
        raise RuntimeError(f"acehip {what} failed ({rc}): {msg.decode() if msg else ''}")


def stream_ptr(stream=None):
    """HIP stream handle of a torch stream (current stream by default)."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return c_void_p(s.cuda_stream)


def dtype_code(t) -> int:
    """ACEHIP_F32 / ACEHIP_BF16 of a tensor (anything else is refused)."""
    import torch
    if t.dtype == torch.float32:
        return ACEHIP_F32
    if t.dtype == torch.bfloat16:
        return ACEHIP_BF16
    raise TypeError(f"acehip: unsupported dtype {t.dtype}")


def ptr(t):
    return c_void_p(t.data_ptr()) if t is not None else None


def shape_arg(shape):
    return (c_int64 * len(shape))(*shape)
