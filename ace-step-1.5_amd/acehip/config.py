"""Model hyper-parameters for the two hot-path networks.

DiT: mirrors the fields of ``AceStepConfig`` the decoder uses
(reference ``acestep/models/base/configuration_acestep_v15.py:148-260``).
VAE: mirrors diffusers ``AutoencoderOobleck`` config fields as consumed by
``acestep/models/mlx/vae_model.py:237-281`` with ACE-Step's hop of 1920
(``acestep/core/generation/handler/conditioning_masks.py:42-43``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class DiTConfig:
    hidden_size: int = 2048
    intermediate_size: int = 6144
    num_hidden_layers: int = 24
    num_attention_heads: int = 16
    num_key_value_heads: int = 8
    head_dim: int = 128
    sliding_window: int = 128
    patch_size: int = 2
    in_channels: int = 192
    audio_acoustic_hidden_dim: int = 64
    rms_norm_eps: float = 1e-6
    rope_theta: float = 1_000_000.0
    layer_types: Optional[List[str]] = None
    # condition encoders (configuration_acestep_v15.py:173-185)
    num_lyric_encoder_hidden_layers: int = 8
    num_timbre_encoder_hidden_layers: int = 4
    num_attention_pooler_hidden_layers: int = 2
    text_hidden_dim: int = 1024
    timbre_hidden_dim: int = 64
    pool_window_size: int = 5

    def __post_init__(self):
        if self.layer_types is None:
            # configuration_acestep_v15.py:250-254 — even index sliding, odd full.  The
            # encoders index the same list by their own layer index (base:399), so it
            # must cover the deepest stack.
            n = max(self.num_hidden_layers, self.num_lyric_encoder_hidden_layers,
                    self.num_timbre_encoder_hidden_layers, self.num_attention_pooler_hidden_layers)
            self.layer_types = [
                "sliding_attention" if (i + 1) % 2 else "full_attention"
                for i in range(n)
            ]

    @property
    def q_dim(self) -> int:
        return self.num_attention_heads * self.head_dim

    @property
    def kv_dim(self) -> int:
        return self.num_key_value_heads * self.head_dim

    def is_sliding(self, layer: int) -> bool:
        return self.layer_types[layer] == "sliding_attention"

    @classmethod
    def tiny(cls, layers: int = 2, window: int = 8) -> "DiTConfig":
        """Reduced-width config used for golden vectors and fast parity tests.

        Keeps head_dim=128 and the 2:1 GQA ratio of the real model so the HIP
        kernels run their production code paths."""
        return cls(hidden_size=256, intermediate_size=512, num_hidden_layers=layers,
                   num_attention_heads=2, num_key_value_heads=1, head_dim=128,
                   sliding_window=window)


@dataclass
class VAEConfig:
    encoder_hidden_size: int = 128
    downsampling_ratios: List[int] = field(default_factory=lambda: [2, 4, 4, 6, 10])
    channel_multiples: List[int] = field(default_factory=lambda: [1, 2, 4, 8, 16])
    decoder_channels: int = 128
    decoder_input_channels: int = 64
    audio_channels: int = 2

    @property
    def hop_length(self) -> int:
        h = 1
        for r in self.downsampling_ratios:
            h *= r
        return h

    @property
    def upsampling_ratios(self) -> List[int]:
        return list(reversed(self.downsampling_ratios))

    def decoder_block_channels(self):
        """[(c_in, c_out, stride)] for the 5 decoder blocks (vae_model.py:205-217)."""
        cm = [1] + list(self.channel_multiples)
        n = len(self.upsampling_ratios)
        out = []
        for i, s in enumerate(self.upsampling_ratios):
            out.append((self.decoder_channels * cm[n - i], self.decoder_channels * cm[n - i - 1], s))
        return out

    def encoder_block_channels(self):
        """[(c_in, c_out, stride)] for the 5 encoder blocks (vae_model.py:160-176)."""
        cm = [1] + list(self.channel_multiples)
        return [(self.encoder_hidden_size * cm[i], self.encoder_hidden_size * cm[i + 1], s)
                for i, s in enumerate(self.downsampling_ratios)]

    @classmethod
    def tiny(cls) -> "VAEConfig":
        """Narrow VAE with the real strides (hop 1920) for fast parity tests."""
        return cls(encoder_hidden_size=128, channel_multiples=[1, 1, 1, 1, 1],
                   decoder_channels=128, decoder_input_channels=64)
