#!/usr/bin/env python3
"""Golden vectors for the Qwen3 text encoder: the reference's
``text_encoder`` is a transformers ``Qwen3Model`` (AutoModel of Qwen3-Embedding-0.6B,
``init_service_loader.py:146-160``), called as ``text_encoder(input_ids=ids,
lyric_attention_mask=None).last_hidden_state`` (``conditioning_embed.py:71-74``).
transformers is a third-party dependency importable in this container (5.15; the
reference pins <4.58): a tiny Qwen3Model with the seeded synthetic weights of
``acehip.weights.synth_text_encoder_weights`` (parity mode; the tests regenerate them)
is run here in fp32 and, cast with ``.to(torch.bfloat16)`` exactly as the reference
loader does, in bf16.  Ids and outputs go to tests/golden/textenc_tiny.safetensors.

usage: python tools/make_golden_text.py
"""
import os
import sys
import torch
from safetensors.torch import save_file
from transformers import Qwen3Config, Qwen3Model

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
from acehip.config import DiTConfig  # noqa: E402
from acehip.weights import synth_text_encoder_weights  # noqa: E402
SEED = 7
CFG = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=3, num_attention_heads=2,
           num_key_value_heads=1, head_dim=128, rms_norm_eps=1e-6, rope_theta=1_000_000.0,
           max_position_embeddings=4096, attention_bias=False, use_sliding_window=False)


def dit_cfg() -> DiTConfig:
    return DiTConfig(hidden_size=CFG["hidden_size"], intermediate_size=CFG["intermediate_size"],
                     num_hidden_layers=CFG["num_hidden_layers"], num_attention_heads=CFG["num_attention_heads"],
                     num_key_value_heads=CFG["num_key_value_heads"], head_dim=CFG["head_dim"],
                     rms_norm_eps=CFG["rms_norm_eps"], rope_theta=CFG["rope_theta"])


def main():
    torch.manual_seed(0)
    cfg = Qwen3Config(**CFG)
    model = Qwen3Model(cfg).eval()
    W = synth_text_encoder_weights(dit_cfg(), CFG["vocab_size"], seed=SEED, mode="parity")
    missing, unexpected = model.load_state_dict(W, strict=False)
    assert not unexpected and all(k.startswith("rotary_emb") for k in missing), (missing, unexpected)
    g = torch.Generator().manual_seed(1)
    out = {}
    for tag, (B, S) in {"a": (2, 37), "b": (1, 150)}.items():
        ids = torch.randint(0, CFG["vocab_size"], (B, S), generator=g)
        out[f"ids_{tag}"] = ids
        with torch.no_grad():
            out[f"out_f32_{tag}"] = model(input_ids=ids, lyric_attention_mask=None).last_hidden_state.contiguous()
    mb = model.to(torch.bfloat16)
    for tag in ("a", "b"):
        with torch.no_grad():
            out[f"out_bf16_{tag}"] = mb(input_ids=out[f"ids_{tag}"]).last_hidden_state.contiguous()
    save_file(out, os.path.join(REPO, "tests", "golden", "textenc_tiny.safetensors"),
              metadata={k: str(v) for k, v in CFG.items()})
    print("wrote", len(out), "tensors")


if __name__ == "__main__":
    main()
