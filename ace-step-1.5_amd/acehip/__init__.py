"""acehip — MI355X (gfx950) implementation of the ACE-Step 1.5 hot path.

DiT flow-matching denoise loop (``AceStepDiTBackend.generate_audio``) and the
Oobleck VAE decode/encode (``OobleckBackend``) behind libacehip.so's C ABI
(include/acehip.h).  See DESIGN.md.
"""
from .config import DiTConfig, VAEConfig  # noqa: F401

__all__ = ["DiTConfig", "VAEConfig"]
