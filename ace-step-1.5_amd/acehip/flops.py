"""Algorithmic work per unit — the denominators of every
roofline fraction bench.py reports."""


def dit_flops_per_row(cfg, S: int, Lenc: int) -> float:
    """Algorithmic FLOPs of one DiT forward per batch row (SURVEY §8d formula)."""
    D, H, KV, hd, F_, L, W_ = (cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                               cfg.head_dim, cfg.intermediate_size, cfg.num_hidden_layers,
                               cfg.sliding_window)
    pairs = sum(min(S - 1, i + W_) - max(0, i - W_) + 1 for i in range(S))
    per_layer = (2 * S * (D * H * hd + 2 * D * KV * hd + H * hd * D) + 2 * S * (2 * D * H * hd)
                 + 2 * S * 3 * D * F_ + 4 * S * Lenc * H * hd)
    n_full = sum(1 for i in range(L) if not cfg.is_sliding(i))
    n_band = L - n_full
    return (L * per_layer + n_full * 4 * S * S * H * hd + n_band * 4 * pairs * H * hd
            + 2 * S * (2 * cfg.in_channels) * D + 2 * S * D * (2 * cfg.audio_acoustic_hidden_dim))


def dit_flops_executed_cfg_song_step(cfg, S: int, Lenc: int, dedup: bool = True) -> float:
    """FLOPs the HIP path actually executes for one CFG step of one song (Bc = 2):
    the reference's algorithmic work of both rows minus what is skipped
    algebraically — the null row's cross-Q projection, cross-attention and cross-O
    GEMM (its output is a per-layer constant, DESIGN §3 "CFG null rows") and, with
    the layer-0 dedup, the second row's proj_in and layer-0 self-attention block
    (both rows are identical until the first cross-attention)."""
    D, H, KV, hd, L, W_ = (cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                           cfg.head_dim, cfg.num_hidden_layers, cfg.sliding_window)
    full = 2 * dit_flops_per_row(cfg, S, Lenc)
    skipped = L * (2 * S * D * H * hd + 4 * S * Lenc * H * hd + 2 * S * H * hd * D)
    if dedup:
        pairs = sum(min(S - 1, i + W_) - max(0, i - W_) + 1 for i in range(S))
        attn0 = 4 * (pairs if cfg.is_sliding(0) else S * S) * H * hd
        skipped += 2 * S * D * (H + 2 * KV) * hd + attn0 + 2 * S * H * hd * D + 2 * S * (2 * cfg.in_channels) * D
    return full - skipped


def vae_decoder_flops(cfg, T: int) -> float:
    """Σ 2·L_out·C_in·C_out·k over the decoder convs."""
    total = 2.0 * T * cfg.decoder_input_channels * cfg.decoder_block_channels()[0][0] * 7
    L = T
    for cin, cout, s in cfg.decoder_block_channels():
        L *= s
        total += 2.0 * L * cin * cout * 2  # ConvT k=2s, each output sees 2 taps
        total += 3 * (2.0 * L * cout * cout * 7 + 2.0 * L * cout * cout)
    total += 2.0 * L * cfg.decoder_channels * cfg.audio_channels * 7
    return total
