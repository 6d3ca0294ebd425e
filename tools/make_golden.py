#!/usr/bin/env python3
"""Generate golden vectors by importing the REFERENCE (this container only).

Runs the reference's own code from ``/root/reference/acestep/models/{base,turbo}``
(read-only, never copied) on small inputs and stores inputs + outputs as
safetensors fixtures under ``tests/golden/``.  Weights are NOT stored: they
are regenerated bit-exactly from ``acehip.weights.synth_dit_weights(cfg,
seed, mode="parity")`` (NumPy PCG64), and a checksum is stored to detect drift.

Fixtures:
  dit_fwd_*.safetensors      one decoder forward (tiny + full-width configs,
                             fp32 + bf16, even/odd T)
  temb_*.safetensors         TimestepEmbedding outputs for schedule values
  adg_*.safetensors          adg_forward on seeded inputs (ADG guidance)
  sampler_*.safetensors      a whole generate_audio (base CFG+APG or ADG / turbo)
                             driven by a deterministic stand-in decoder that
                             records every (x, t, vt) — pins schedules, APG,
                             momentum, Euler/x0 arithmetic bit-exactly.

``vector_quantize_pytorch`` (absent here) is stubbed; its ResidualFSQ is only
used by the audio tokenizer whose output is discarded when is_covers=0
(reference base:1645-1649).
"""
from __future__ import annotations

import json
import os
import sys
import types

import torch
from safetensors.torch import save_file

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]
OUT = os.path.join(REPO, "tests", "golden")

from acehip.config import DiTConfig  # noqa: E402
from acehip.weights import synth_dit_weights, synth_null_condition  # noqa: E402


def _stub_vq():
    m = types.ModuleType("vector_quantize_pytorch")

    class ResidualFSQ(torch.nn.Module):
        def __init__(self, *a, **k):
            super().__init__()

        def forward(self, x):
            return x, None

    m.ResidualFSQ = ResidualFSQ
    sys.modules["vector_quantize_pytorch"] = m


def _import_ref(variant: str):
    _stub_vq()
    d = f"/root/reference/acestep/models/{variant}"
    for k in list(sys.modules):
        if k.startswith(("configuration_acestep_v15", "modeling_acestep_v15", "apg_guidance")):
            del sys.modules[k]
    sys.path.insert(0, d)
    try:
        import configuration_acestep_v15 as C
        # the sft variant ships its modeling file under the base name
        mod = __import__(f"modeling_acestep_v15_{'base' if variant == 'sft' else variant}")
    finally:
        sys.path.remove(d)
    return C, mod


def ref_config(C, cfg: DiTConfig, **extra):
    rc = C.AceStepConfig(hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
                         num_hidden_layers=cfg.num_hidden_layers,
                         num_attention_heads=cfg.num_attention_heads,
                         num_key_value_heads=cfg.num_key_value_heads, head_dim=cfg.head_dim,
                         sliding_window=cfg.sliding_window, **extra)
    rc._attn_implementation = "sdpa"
    return rc


def checksum(W) -> float:
    return float(sum(float(v.double().abs().sum()) for v in W.values()))


def gen_forward(M, C, name, cfg: DiTConfig, B, T, Lenc, dtype, seed, t_vals, tr_vals):
    rc = ref_config(C, cfg)
    model = M.AceStepDiTModel(rc).eval()
    W = synth_dit_weights(cfg, seed=seed, mode="parity", workers=8)
    missing, unexpected = model.load_state_dict(W, strict=False)
    assert not unexpected and all("rotary" in k for k in missing), (missing, unexpected)
    model = model.to(dtype)
    g = torch.Generator().manual_seed(1234 + T)
    xt = torch.randn(B, T, 64, generator=g).to(dtype)
    ctx = torch.randn(B, T, 128, generator=g).to(dtype)
    ctx[..., 64:] = (ctx[..., 64:] > 0).to(dtype)  # chunk-mask-like channels
    enc = torch.randn(B, Lenc, cfg.hidden_size, generator=g).to(dtype)
    t = torch.tensor(t_vals, dtype=dtype)
    tr = torch.tensor(tr_vals, dtype=dtype)
    with torch.no_grad():
        out = model(hidden_states=xt, timestep=t, timestep_r=tr, attention_mask=None,
                    encoder_hidden_states=enc, encoder_attention_mask=None,
                    context_latents=ctx, use_cache=False)[0]
    save_file({"xt": xt, "ctx": ctx, "enc": enc, "t": t, "t_r": tr, "vt": out.contiguous()},
              os.path.join(OUT, f"dit_fwd_{name}.safetensors"))
    return {"cfg": cfg.__dict__, "B": B, "T": T, "Lenc": Lenc, "dtype": str(dtype),
            "seed": seed, "weights_checksum": checksum(W)}


def gen_temb(M, C, cfg, dtype, seed):
    rc = ref_config(C, cfg)
    model = M.AceStepDiTModel(rc).eval()
    model.load_state_dict(synth_dit_weights(cfg, seed=seed, mode="parity"), strict=False)
    model = model.to(dtype)
    t = torch.tensor([1.0, 0.9545454545454546, 0.75, 0.5, 0.3, 0.125, 0.0], dtype=dtype)
    with torch.no_grad():
        temb, proj = model.time_embed(t)
    save_file({"t": t, "temb": temb.contiguous(), "proj": proj.contiguous()},
              os.path.join(OUT, f"temb_{str(dtype).split('.')[-1]}.safetensors"))


class _Recorder(torch.nn.Module):
    """Stand-in decoder: deterministic, depends on x, t, encoder states and
    context so cond/uncond halves differ; records every call."""

    def __init__(self):
        super().__init__()
        self.calls = []

    def forward(self, hidden_states, timestep, timestep_r, attention_mask, encoder_hidden_states,
                encoder_attention_mask, context_latents, use_cache=True, past_key_values=None, **kw):
        x = hidden_states
        e = torch.tanh(encoder_hidden_states.float().mean(1, keepdim=True)[..., :64])
        v = (0.6 * x.float() + 0.4 * e + 0.1 * context_latents[..., :64].float()
             * timestep.float()[:, None, None] + 0.05 * torch.sin(3.0 * x.float()))
        v = v.to(x.dtype)
        self.calls.append((x.clone(), timestep.clone(), v.clone(), encoder_hidden_states.clone(),
                           context_latents.clone()))
        return (v, past_key_values)


def gen_sampler(variant, name, dtype, B, T, **gen_kw):
    C, M = _import_ref(variant)
    cfg = DiTConfig.tiny(layers=1)
    rc = ref_config(C, cfg, num_lyric_encoder_hidden_layers=1, num_timbre_encoder_hidden_layers=1,
                    num_attention_pooler_hidden_layers=1, num_audio_decoder_hidden_layers=1)
    torch.manual_seed(0)
    model = M.AceStepConditionGenerationModel(rc).eval().to(dtype)
    with torch.no_grad():
        model.null_condition_emb.copy_(synth_null_condition(cfg, seed=7).to(dtype))
    rec = _Recorder()
    model.decoder = rec
    g = torch.Generator().manual_seed(99)
    Lt, Ll = 6, 9
    kw = dict(
        text_hidden_states=torch.randn(B, Lt, 1024, generator=g).to(dtype),
        text_attention_mask=torch.ones(B, Lt, dtype=torch.long),
        lyric_hidden_states=torch.randn(B, Ll, 1024, generator=g).to(dtype),
        lyric_attention_mask=torch.ones(B, Ll, dtype=torch.long),
        refer_audio_acoustic_hidden_states_packed=torch.randn(B, 750, 64, generator=g).to(dtype),
        refer_audio_order_mask=torch.arange(B, dtype=torch.long),
        src_latents=torch.randn(B, T, 64, generator=g).to(dtype),
        chunk_masks=torch.ones(B, T, 64, dtype=dtype),
        is_covers=torch.zeros(B, dtype=torch.long),
        silence_latent=torch.randn(1, T, 64, generator=g).to(dtype),
        seed=list(range(B)), use_progress_bar=False,
    )
    if gen_kw.get("audio_cover_strength", 1.0) < 1.0:
        kw["non_cover_text_hidden_states"] = torch.randn(B, Lt, 1024, generator=g).to(dtype)
        kw["non_cover_text_attention_mask"] = torch.ones(B, Lt, dtype=torch.long)
    kw.update(gen_kw)
    # the SDE branch re-noises with the unseeded global RNG (base:1777 randn_like,
    # turbo:1984): record every draw so a replay can inject the same noise
    noise_draws = []
    orig_randn_like = torch.randn_like

    def randn_like(x, *a, **k):
        n = orig_randn_like(x, *a, **k)
        noise_draws.append(n.clone())
        return n
    torch.randn_like = randn_like
    try:
        with torch.no_grad():
            res = model.generate_audio(**kw)
    finally:
        torch.randn_like = orig_randn_like
    tensors = {"target_latents": res["target_latents"].contiguous()}
    for i, (x, t, v, e, c) in enumerate(rec.calls):
        tensors[f"x_{i}"] = x
        tensors[f"t_{i}"] = t
        tensors[f"vt_{i}"] = v
        tensors[f"enc_{i}"] = e
        tensors[f"ctx_{i}"] = c
    for i, n in enumerate(noise_draws):
        tensors[f"noise_{i}"] = n
    tensors["enc"] = rec.calls[0][3].clone()
    tensors["ctx"] = rec.calls[0][4].clone()
    tensors["src_latents"] = kw["src_latents"].clone()
    tensors["silence_latent"] = kw["silence_latent"].clone()
    save_file(tensors, os.path.join(OUT, f"sampler_{name}.safetensors"))
    meta = {k: (v if isinstance(v, (int, float, str, bool, list)) else
                (v.tolist() if isinstance(v, torch.Tensor) else None)) for k, v in gen_kw.items()}
    return {"variant": variant, "dtype": str(dtype), "B": B, "T": T, "n_calls": len(rec.calls),
            "n_noise": len(noise_draws), "kwargs": meta}


def gen_adg_direct(name, B, T, seed, sigmas, guidance):
    """adg_forward (apg_guidance.py:107-180) called directly on seeded bf16
    inputs — includes rows where cond == uncond (θ = 0 branch) and a fully
    aligned row pair (sin θ ≤ 1e-3 branch)."""
    _import_ref("base")
    import apg_guidance as ag
    g = torch.Generator().manual_seed(seed)
    tensors = {}
    for i, sg in enumerate(sigmas):
        x = torch.randn(B, T, 64, generator=g).bfloat16()
        c = torch.randn(B, T, 64, generator=g).bfloat16()
        u = (c.float() + 0.3 * torch.randn(B, T, 64, generator=g)).bfloat16()
        u[:, 3] = (c[:, 3].float() * 1.0005).bfloat16()      # nearly parallel hats
        s = torch.tensor(sg, dtype=torch.bfloat16)
        out = ag.adg_forward(latents=x, noise_pred_cond=c, noise_pred_uncond=u, sigma=s,
                             guidance_scale=guidance)
        tensors.update({f"x_{i}": x, f"cond_{i}": c, f"uncond_{i}": u, f"sigma_{i}": s.reshape(1),
                        f"out_{i}": out.contiguous()})
    save_file(tensors, os.path.join(OUT, f"adg_{name}.safetensors"))
    return {"B": B, "T": T, "sigmas": sigmas, "guidance": guidance}


def condenc_config(width: str) -> DiTConfig:
    if width == "tiny":
        return DiTConfig(hidden_size=256, intermediate_size=512, num_hidden_layers=4, num_attention_heads=2,
                         num_key_value_heads=1, head_dim=128, sliding_window=8,
                         num_lyric_encoder_hidden_layers=3, num_timbre_encoder_hidden_layers=2,
                         num_attention_pooler_hidden_layers=2)
    return DiTConfig(num_hidden_layers=2, num_lyric_encoder_hidden_layers=2, num_timbre_encoder_hidden_layers=1,
                     num_attention_pooler_hidden_layers=1)


def gen_condenc(name, width, dtype, seed):
    """AceStepConditionEncoder.forward (base:1527-1554) on ragged padded inputs:
    lyric rows with padding (and, with the 8-wide band of the tiny config, padded
    query rows that see NO admissible key — the uniform-softmax case), text rows
    with padding, 3 packed timbre references for 2 songs (order [0, 1, 1])."""
    from acehip.weights import synth_condenc_weights
    C, M = _import_ref("base")
    cfg = condenc_config(width)
    rc = ref_config(C, cfg, num_lyric_encoder_hidden_layers=cfg.num_lyric_encoder_hidden_layers,
                    num_timbre_encoder_hidden_layers=cfg.num_timbre_encoder_hidden_layers,
                    num_attention_pooler_hidden_layers=cfg.num_attention_pooler_hidden_layers)
    model = M.AceStepConditionEncoder(rc).eval()
    W = synth_condenc_weights(cfg, seed=seed, mode="parity")
    missing, unexpected = model.load_state_dict(W, strict=False)
    assert not unexpected and all("rotary" in k for k in missing), (missing, unexpected)
    model = model.to(dtype)
    g = torch.Generator().manual_seed(seed + 1)
    B, Lt, Ll, Nref, Tref = 2, 7, 41, 3, 30
    text = torch.randn(B, Lt, cfg.text_hidden_dim, generator=g).to(dtype)
    tmask = torch.ones(B, Lt, dtype=torch.long)
    tmask[1, 4:] = 0
    lyric = torch.randn(B, Ll, cfg.text_hidden_dim, generator=g).to(dtype)
    lmask = torch.ones(B, Ll, dtype=torch.long)
    lmask[1, 17:] = 0
    lmask[0, 39:] = 0
    refer = torch.randn(Nref, Tref, cfg.timbre_hidden_dim, generator=g).to(dtype)
    order = torch.tensor([0, 1, 1], dtype=torch.long)
    with torch.no_grad():
        lyr = model.lyric_encoder(inputs_embeds=lyric, attention_mask=lmask).last_hidden_state
        tim, tim_mask = model.timbre_encoder(refer, order)
        enc, enc_mask = model(text_hidden_states=text, text_attention_mask=tmask, lyric_hidden_states=lyric,
                              lyric_attention_mask=lmask, refer_audio_acoustic_hidden_states_packed=refer,
                              refer_audio_order_mask=order)
    save_file({"text": text, "text_mask": tmask, "lyric": lyric, "lyric_mask": lmask, "refer": refer,
               "order": order, "lyric_out": lyr.contiguous(), "timbre_out": tim.contiguous(),
               "timbre_mask": tim_mask.contiguous(), "enc": enc.contiguous(),
               "enc_mask": enc_mask.to(torch.uint8).contiguous()},
              os.path.join(OUT, f"condenc_{name}.safetensors"))
    return {"width": width, "cfg": cfg.__dict__, "dtype": str(dtype), "seed": seed,
            "weights_checksum": checksum(W)}


class _FsqRestated(torch.nn.Module):
    """Stand-in for vector_quantize_pytorch.ResidualFSQ (absent here): the oracle's
    restatement of its published algorithm, so the tokenizer fixture pins the
    reference's projection + attention pooler around it (the FSQ part itself is
    parity-unpinned)."""

    def __init__(self, dim, levels, num_quantizers, **kw):
        super().__init__()
        self.project_in = torch.nn.Linear(dim, len(levels))
        self.project_out = torch.nn.Linear(len(levels), dim)

    def forward(self, x):
        from oracle.condenc_oracle import fsq_quantize
        codes, idx = fsq_quantize(self.project_in(x))
        return self.project_out(codes), idx.unsqueeze(-1)


def gen_tokenizer(name, dtype, seed):
    """AttentionPooler (base:734-859), AceStepAudioTokenizer (base:1181-1223, with
    the restated FSQ) and AudioTokenDetokenizer (base:862-994) of the reference."""
    from acehip.weights import synth_tokenizer_weights
    C, M = _import_ref("base")
    M.ResidualFSQ = _FsqRestated
    cfg = condenc_config("tiny")
    rc = ref_config(C, cfg, num_lyric_encoder_hidden_layers=cfg.num_lyric_encoder_hidden_layers,
                    num_timbre_encoder_hidden_layers=cfg.num_timbre_encoder_hidden_layers,
                    num_attention_pooler_hidden_layers=cfg.num_attention_pooler_hidden_layers, fsq_dim=cfg.hidden_size)
    W = synth_tokenizer_weights(cfg, seed=seed, mode="parity")
    tok = M.AceStepAudioTokenizer(rc).eval()
    det = M.AudioTokenDetokenizer(rc).eval()
    mt, ut = tok.load_state_dict({k[len("tokenizer."):]: v for k, v in W.items() if k.startswith("tokenizer.")},
                                 strict=False)
    md, ud = det.load_state_dict({k[len("detokenizer."):]: v for k, v in W.items() if k.startswith("detokenizer.")},
                                 strict=False)
    assert not ut and not ud and all("rotary" in k for k in mt + md), (mt, ut, md, ud)
    tok, det = tok.to(dtype), det.to(dtype)
    g = torch.Generator().manual_seed(seed + 1)
    N, T = 2, 30
    x = torch.randn(N, T, cfg.audio_acoustic_hidden_dim, generator=g).to(dtype)
    pooled_in = torch.randn(N, T // 5, 5, cfg.hidden_size, generator=g).to(dtype)
    det_in = torch.randn(N, T // 5, cfg.hidden_size, generator=g).to(dtype)
    with torch.no_grad():
        pooled = tok.attention_pooler(pooled_in)
        quant, idx = tok.tokenize(x)
        det_out = det(det_in)
        hints = det(quant)
    save_file({"x": x, "pooled_in": pooled_in, "pooled": pooled.contiguous(), "quantized": quant.contiguous(),
               "indices": idx.contiguous(), "det_in": det_in, "det_out": det_out.contiguous(),
               "hints": hints.contiguous()}, os.path.join(OUT, f"tokenizer_{name}.safetensors"))
    return {"cfg": cfg.__dict__, "dtype": str(dtype), "seed": seed, "weights_checksum": checksum(W),
            "note": "ResidualFSQ replaced by the oracle restatement (vector_quantize_pytorch absent): quantizer parity unpinned"}


def main_only(which):
    """Add fixtures to an existing manifest without regenerating the rest."""
    torch.set_num_threads(8)
    mpath = os.path.join(OUT, "manifest.json")
    manifest = json.load(open(mpath))
    bf = torch.bfloat16
    if "adg" in which:
        manifest["adg"] = {"direct": gen_adg_direct("direct", 1, 48, 5, [1.0, 0.75, 0.30078125, 0.05],
                                                    7.0)}
        manifest["sampler"]["base_s8_adg"] = gen_sampler("base", "base_s8_adg", bf, 1, 40, infer_steps=8,
                                                         shift=3.0, diffusion_guidance_sale=7.0,
                                                         use_adg=True)
    if "sampler2" in which:
        # the branches round 1 left without a GPU replay: cover-noise truncation
        # (base:1879-1902, turbo:1922-1936), the cover -> non-cover switch
        # (base:1836-1856,1916-1927; turbo:1892-1956), SDE re-noise (base:1968-1973,
        # turbo:1980-1984) with the unseeded draws recorded, sft custom timesteps
        # (sft:1866-1868)
        sm = manifest["sampler"]
        sm["base_s8_cover"] = gen_sampler("base", "base_s8_cover", bf, 2, 40, infer_steps=8, shift=3.0,
                                          diffusion_guidance_sale=7.0, cover_noise_strength=0.35)
        sm["base_s8_acs"] = gen_sampler("base", "base_s8_acs", bf, 1, 40, infer_steps=8, shift=3.0,
                                        diffusion_guidance_sale=7.0, audio_cover_strength=0.5)
        sm["base_s8_sde"] = gen_sampler("base", "base_s8_sde", bf, 2, 40, infer_steps=8, shift=3.0,
                                        diffusion_guidance_sale=7.0, infer_method="sde")
        sm["base_s10_cover_acs_sde"] = gen_sampler("base", "base_s10_cover_acs_sde", bf, 1, 32, infer_steps=10,
                                                   shift=2.0, diffusion_guidance_sale=5.0, cover_noise_strength=0.5,
                                                   audio_cover_strength=0.6, infer_method="sde")
        sm["turbo_cover_acs"] = gen_sampler("turbo", "turbo_cover_acs", bf, 1, 40, shift=3.0,
                                            cover_noise_strength=0.3, audio_cover_strength=0.5)
        sm["turbo_sde"] = gen_sampler("turbo", "turbo_sde", bf, 2, 40, shift=1.0, infer_method="sde")
        sm["sft_timesteps"] = gen_sampler("sft", "sft_timesteps", bf, 1, 40, diffusion_guidance_sale=7.0,
                                          shift=3.0, timesteps=torch.tensor([1.0, 0.9, 0.7, 0.5, 0.3, 0.1, 0.0]))
    if "sampler_fp32" in which:
        # the fp32 parity mode of the samplers (the reference's fp32 path off cuda/xpu)
        f32 = torch.float32
        sm = manifest["sampler"]
        sm["base_s8_sh3_fp32"] = gen_sampler("base", "base_s8_sh3_fp32", f32, 2, 40, infer_steps=8, shift=3.0,
                                             diffusion_guidance_sale=7.0)
        sm["base_s8_adg_fp32"] = gen_sampler("base", "base_s8_adg_fp32", f32, 1, 40, infer_steps=8, shift=3.0,
                                             diffusion_guidance_sale=7.0, use_adg=True)
        sm["turbo_sh3_fp32"] = gen_sampler("turbo", "turbo_sh3_fp32", f32, 2, 40, shift=3.0)
    if "long" in which:
        # full width with S > 2W+1 so the ±128 band of the even layers is pinned at full
        # width against the reference (base:56-135, :1378-1447); odd T (pad + crop)
        full2 = DiTConfig(num_hidden_layers=2)
        C, M = _import_ref("base")
        for dt in (torch.float32, torch.bfloat16):
            tag = str(dt).split(".")[-1]
            manifest["forward"][f"full2_long_{tag}"] = gen_forward(M, C, f"full2_long_{tag}", full2, 2, 641, 48, dt,
                                                                  22, [0.5, 0.5], [0.5, 0.5])
    if "full24" in which:
        # the real 24-layer decoder (configuration_acestep_v15.py:148-260; the layer loop
        # base:1463-1485) at the size SURVEY §8c calibrated its tolerance on: T = 500,
        # Lenc = 200, one broadcast timestep for both rows (the CFG production layout)
        full24 = DiTConfig()
        assert full24.num_hidden_layers == 24
        C, M = _import_ref("base")
        for dt in (torch.float32, torch.bfloat16):
            tag = str(dt).split(".")[-1]
            manifest["forward"][f"full24_{tag}"] = gen_forward(M, C, f"full24_{tag}", full24, 2, 500, 200, dt,
                                                              51, [0.6328125, 0.6328125], [0.6328125, 0.6328125])
    if "tokenizer" in which:
        manifest["tokenizer"] = {f"tiny_{str(dt).split('.')[-1]}": gen_tokenizer(f"tiny_{str(dt).split('.')[-1]}", dt, 41)
                                 for dt in (torch.float32, torch.bfloat16)}
    if "condenc" in which:
        ce = {}
        for width in ("tiny", "full"):
            for dt in (torch.float32, torch.bfloat16):
                tag = f"{width}_{str(dt).split('.')[-1]}"
                ce[tag] = gen_condenc(tag, width, dt, 31 if width == "tiny" else 32)
        manifest["condenc"] = ce
    with open(mpath, "w") as f:
        json.dump(manifest, f, indent=1, default=str)
    print("updated", mpath)


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(8)
    manifest = {"generator": "tools/make_golden.py", "reference": "/root/reference (read-only import)",
                "torch": torch.__version__}
    import transformers
    manifest["transformers"] = transformers.__version__
    C, M = _import_ref("base")
    fw = {}
    tiny = DiTConfig.tiny(layers=4, window=8)
    for dt in (torch.float32, torch.bfloat16):
        tag = str(dt).split(".")[-1]
        fw[f"tiny_{tag}"] = gen_forward(M, C, f"tiny_{tag}", tiny, 2, 50, 20, dt, 11,
                                        [0.75, 0.3], [0.75, 0.3])
        fw[f"tiny_odd_{tag}"] = gen_forward(M, C, f"tiny_odd_{tag}", tiny, 2, 49, 13, dt, 12,
                                            [1.0, 0.5], [0.25, 0.5])
        gen_temb(M, C, tiny, dt, 11)
    full2 = DiTConfig(num_hidden_layers=2)
    for dt in (torch.float32, torch.bfloat16):
        tag = str(dt).split(".")[-1]
        fw[f"full2_{tag}"] = gen_forward(M, C, f"full2_{tag}", full2, 2, 64, 16, dt, 21,
                                         [0.9, 0.9], [0.9, 0.9])
    manifest["forward"] = fw
    sm = {}
    bf = torch.bfloat16
    sm["base_s8_sh3"] = gen_sampler("base", "base_s8_sh3", bf, 2, 40, infer_steps=8, shift=3.0,
                                    diffusion_guidance_sale=7.0)
    sm["base_s27_sh3"] = gen_sampler("base", "base_s27_sh3", bf, 1, 40, infer_steps=27, shift=3.0,
                                     diffusion_guidance_sale=7.0)
    sm["base_s60_sh3"] = gen_sampler("base", "base_s60_sh3", bf, 1, 24, infer_steps=60, shift=3.0,
                                     diffusion_guidance_sale=7.0)
    sm["base_s10_sh1_interval"] = gen_sampler("base", "base_s10_sh1_interval", bf, 2, 32,
                                              infer_steps=10, shift=1.0, diffusion_guidance_sale=4.0,
                                              cfg_interval_start=0.3, cfg_interval_end=0.8)
    sm["base_s8_nocfg_fp32"] = gen_sampler("base", "base_s8_nocfg_fp32", torch.float32, 2, 32,
                                           infer_steps=8, shift=2.0, diffusion_guidance_sale=1.0)
    sm["turbo_sh3"] = gen_sampler("turbo", "turbo_sh3", bf, 2, 40, shift=3.0)
    sm["turbo_sh2"] = gen_sampler("turbo", "turbo_sh2", bf, 1, 40, shift=2.2)
    sm["turbo_custom"] = gen_sampler("turbo", "turbo_custom", bf, 1, 40,
                                     timesteps=torch.tensor([0.97, 0.76, 0.5, 0.26, 0.0]))
    manifest["sampler"] = sm
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, default=str)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--only":
        main_only(sys.argv[2].split(","))
    else:
        main()
