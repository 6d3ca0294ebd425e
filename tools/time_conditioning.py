#!/usr/bin/env python3
"""Time rank 0's per-batch conditioning of the song-parallel pipeline on one GPU (verdict r05
item 5): for a batch of B songs at the 240 s bench shapes, what ``SongParallelPipeline.generate``
runs before the scatter — the Qwen3 text encoder (128 tokens) + lyric table lookup (512 tokens),
``prepare_condition`` (lyric encoder 8 layers, timbre encoder 4 layers, pack_sequences) over
the batch, and ``prepare_noise`` — serially (the current critical path) and, for comparison,
the per-song DiT + decode it precedes.  Prints one JSON line per B."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]

import torch  # noqa: E402

from acehip.condition import ConditionEncoder, HipPrepareCondition, TextEncoder  # noqa: E402
from acehip.config import DiTConfig  # noqa: E402
from acehip.dit import prepare_noise  # noqa: E402
from acehip.weights import synth_condenc_weights, synth_text_encoder_weights  # noqa: E402

QWEN3_VOCAB = 151669


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = DiTConfig()
    T, Lt, Ll, Bmax = 6000, 128, 512, 8
    ce = ConditionEncoder(cfg, 0, max_batch=Bmax, max_lyric=Ll, max_refs=Bmax, max_ref_frames=750)
    ce.load(synth_condenc_weights(cfg, seed=0, mode="bench", device=dev, dtype=torch.bfloat16, backend="torch"))
    prep = HipPrepareCondition(ce)
    te_cfg = DiTConfig(**TextEncoder.QWEN3_06B)
    te = TextEncoder(te_cfg, 0, max_batch=Bmax, max_tokens=Lt)
    te.load(synth_text_encoder_weights(te_cfg, QWEN3_VOCAB, seed=0, mode="bench", device=dev, dtype=torch.bfloat16,
                                       backend="torch"))
    g = torch.Generator(device=dev).manual_seed(0)
    text_ids = torch.randint(0, QWEN3_VOCAB, (1, Lt), device=dev, generator=g)
    lyric_ids = torch.randint(0, QWEN3_VOCAB, (1, Ll), device=dev, generator=g)
    refer = torch.randn(1, 750, cfg.timbre_hidden_dim, device=dev, generator=g).bfloat16()
    src = torch.randn(1, T, 64, device=dev, generator=g).bfloat16()
    chunk = torch.ones(1, T, 64, device=dev).bfloat16()

    def once(B):
        e = lambda t: t.expand(B, *t.shape[1:]).contiguous()  # noqa: E731
        th = te(input_ids=e(text_ids), lyric_attention_mask=None).last_hidden_state
        lh = te.embed_tokens(e(lyric_ids))
        enc, _, ctx = prep(text_hidden_states=th, text_attention_mask=torch.ones(B, Lt, device=dev, dtype=torch.long),
                           lyric_hidden_states=lh, lyric_attention_mask=torch.ones(B, Ll, device=dev, dtype=torch.long),
                           refer_audio_acoustic_hidden_states_packed=e(refer),
                           refer_audio_order_mask=torch.arange(B, device=dev, dtype=torch.long),
                           hidden_states=e(src), attention_mask=None, silence_latent=None, src_latents=e(src),
                           chunk_masks=e(chunk), is_covers=torch.zeros(B, device=dev, dtype=torch.long))
        noise = prepare_noise((B, T, 64), dev, torch.bfloat16, list(range(B)))
        return enc, ctx, noise

    for B in (1, 2, 4, 8):
        for _ in range(2):
            once(B)
        torch.cuda.synchronize()
        n = 5
        t0 = time.perf_counter()
        for _ in range(n):
            once(B)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / n * 1e3
        print(json.dumps({"B": B, "conditioning_ms": round(ms, 2), "per_song_ms": round(ms / B, 2)}), flush=True)


if __name__ == "__main__":
    main()
