"""GPU test of the drop-in itself: ``acehip.integration.install()`` on a
handler-shaped stub whose modules carry the reference's state-dict names and
synthetic weights (no reference code runs: the stub's own ``generate_audio`` /
``prepare_condition`` / ``vae.decode`` / ``tiled_decode`` raise if reached).

The handler is driven the way the reference drives it:
  * ``handler.model.prepare_condition(...)`` as ``_execute_service_generate_diffusion``
    calls it (service_generate_execute.py:123-142), then
  * ``handler.model.generate_audio(**kwargs)`` — both calls' kwargs rebuilt from
    ``tests/golden/seam_calls.json``, which ``tools/record_seam.py`` recorded by running the
    reference's own ``_build_service_generate_kwargs`` / ``_execute_service_generate_diffusion``
    (service_generate_execute.py:62-196) against a recording model — under
    ``torch.inference_mode()`` (:121),
  * ``handler.tiled_decode(latents[B, 64, T])`` (generate_music_decode.py:164),
  * the LoRA lifecycle methods (handler/lora/lifecycle.py:164-289) followed by a
    forward that must equal the oracle on the merged weights W + ΔW.
"""
from types import SimpleNamespace

import pytest
import torch

from conftest import cosine, rel_l2
from seam_spec import build_calls

from acehip.config import DiTConfig, VAEConfig
from acehip.weights import synth_condenc_weights, synth_dit_weights, synth_null_condition, synth_vae_weights
from oracle import condenc_oracle, dit_oracle

pytestmark = pytest.mark.gpu


def module_tree(sd, root=None):
    """nn.Module tree whose state_dict() has exactly the given names."""
    root = root if root is not None else torch.nn.Module()
    for name, t in sd.items():
        *path, leaf = name.split(".")
        m = root
        for p in path:
            if p not in m._modules:
                m.add_module(p, torch.nn.Module())
            m = m._modules[p]
        m.register_parameter(leaf, torch.nn.Parameter(t, requires_grad=False))
    return root


def _cfg():
    return DiTConfig(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=2,
                     num_key_value_heads=1, head_dim=128, sliding_window=8, num_lyric_encoder_hidden_layers=2,
                     num_timbre_encoder_hidden_layers=1, num_attention_pooler_hidden_layers=1)


class StubModel(torch.nn.Module):
    """AceStepConditionGenerationModel-shaped: decoder / encoder sub-modules with the
    reference names, null_condition_emb, an HF-style config, and the reference's
    base-variant generate_audio signature (no ``timesteps``)."""

    def __init__(self, cfg, dev):
        super().__init__()
        self.W = {k: v.to(dev, torch.bfloat16) for k, v in synth_dit_weights(cfg, seed=3, mode="parity").items()}
        self.CE = {k: v.to(dev, torch.bfloat16) for k, v in synth_condenc_weights(cfg, seed=4, mode="parity").items()}
        self.decoder = module_tree(self.W)
        self.encoder = module_tree(self.CE)
        self.null_condition_emb = torch.nn.Parameter(
            synth_null_condition(cfg, seed=5).to(dev, torch.bfloat16), requires_grad=False)
        self.config = SimpleNamespace(**cfg.__dict__, is_turbo=False, model_version="base")
        self.tokenizer = self.detokenizer = None

    def prepare_condition(self, **kw):
        raise AssertionError("the reference prepare_condition ran")

    def generate_audio(self, text_hidden_states, text_attention_mask, lyric_hidden_states, lyric_attention_mask,
                       refer_audio_acoustic_hidden_states_packed, refer_audio_order_mask, src_latents, chunk_masks,
                       is_covers, silence_latent=None, attention_mask=None, seed=None, infer_method="ode",
                       use_cache=True, infer_steps=30, diffusion_guidance_sale=7.0, audio_cover_strength=1.0,
                       non_cover_text_hidden_states=None, non_cover_text_attention_mask=None, cfg_interval_start=0.0,
                       cfg_interval_end=1.0, precomputed_lm_hints_25Hz=None, audio_codes=None,
                       use_progress_bar=True, use_adg=False, shift=1.0, cover_noise_strength=0.0, **kwargs):
        raise AssertionError("the reference generate_audio ran")


class StubVae(torch.nn.Module):
    """diffusers AutoencoderOobleck-shaped: config + weight-normed state dict."""

    def __init__(self, vcfg, dev):
        super().__init__()
        self.Wv = synth_vae_weights(vcfg, seed=6, mode="parity", with_encoder=True)
        module_tree({k: v.to(dev, torch.bfloat16) for k, v in self.Wv.items()}, self)
        self.config = SimpleNamespace(encoder_hidden_size=vcfg.encoder_hidden_size,
                                      downsampling_ratios=vcfg.downsampling_ratios,
                                      channel_multiples=vcfg.channel_multiples,
                                      decoder_channels=vcfg.decoder_channels,
                                      decoder_input_channels=vcfg.decoder_input_channels,
                                      audio_channels=vcfg.audio_channels)
        self.dtype = torch.bfloat16

    def decode(self, z):
        raise AssertionError("the reference VAE decode ran")

    def encode(self, x):
        raise AssertionError("the reference VAE encode ran")


class LoraLinear(torch.nn.Module):
    """PEFT LoraLayer shape (base_layer + lora_A/B + scaling, get_delta_weight)."""

    def __init__(self, base, r, scale, dev, seed):
        super().__init__()
        self.base_layer = base
        out_f, in_f = base.weight.shape
        g = torch.Generator().manual_seed(seed)
        self.lora_A = torch.nn.ParameterDict({"default": torch.nn.Parameter(
            (torch.randn(r, in_f, generator=g) * 0.3).to(dev, torch.bfloat16), requires_grad=False)})
        self.lora_B = torch.nn.ParameterDict({"default": torch.nn.Parameter(
            (torch.randn(out_f, r, generator=g) * 0.3).to(dev, torch.bfloat16), requires_grad=False)})
        self.scaling = {"default": scale}
        self.active_adapters = ["default"]
        self.merged = False
        self.disable_adapters = False

    def get_delta_weight(self, a):
        return (self.lora_B[a].float() @ self.lora_A[a].float()) * self.scaling[a]


class StubHandler:
    def __init__(self, dev):
        self.device = str(dev)
        self.dtype = torch.bfloat16
        self.model = StubModel(_cfg(), dev)
        self.vae = StubVae(VAEConfig.tiny(), dev)
        self.text_encoder = None
        self.lora_targets = ["layers.0.self_attn.q_proj", "layers.1.mlp.down_proj"]

    def tiled_decode(self, latents, chunk_size=None, overlap=64, offload_wav_to_cpu=None):
        raise AssertionError("the reference tiled_decode ran")

    def tiled_encode(self, audio, chunk_size=None, overlap=None, offload_latent_to_cpu=True):
        raise AssertionError("the reference tiled_encode (30 s chunk loop) ran")

    offload_policy = False

    def _should_offload_wav_to_cpu(self):          # memory_utils.py:85-103
        return self.offload_policy

    # LoRA lifecycle (handler/lora/lifecycle.py): adapters wrap decoder Linears
    def add_lora(self, path="synthetic", scale=1.0):
        dec = self.model.decoder
        for i, name in enumerate(self.lora_targets):
            *parent, leaf = name.split(".")
            m = dec
            for p in parent:
                m = m._modules[p]
            m._modules[leaf] = LoraLinear(m._modules[leaf], 4, scale, self.model.null_condition_emb.device, 10 + i)
        return "ok"

    def set_lora_scale(self, scale):
        for _, mod in self.model.decoder.named_modules():
            if isinstance(mod, LoraLinear):
                mod.scaling["default"] = scale
        return "ok"

    def unload_lora(self):
        dec = self.model.decoder
        for name in self.lora_targets:
            *parent, leaf = name.split(".")
            m = dec
            for p in parent:
                m = m._modules[p]
            if isinstance(m._modules[leaf], LoraLinear):
                m._modules[leaf] = m._modules[leaf].base_layer
        return "ok"


@pytest.fixture
def installed(gpu_device):
    from acehip.integration import install
    h = StubHandler(gpu_device)
    out = install(h, max_seconds=4.0, max_batch=2, text_encoder=False)
    yield h, out
    out["dit"].rt.close()
    out["vae"].close()


def test_install_drives_handler_calls(gpu_device, installed):
    from acehip.condition import ConditionEncoder, HipPrepareCondition
    from acehip.dit import AceStepDiTBackend, DiTRuntime
    h, out = installed
    # the calls the reference's own seam makes into self.model for one request, rebuilt from the
    # spec tools/record_seam.py recorded by running service_generate_execute.py:62-196
    payload, silence, calls = build_calls("base_seed_list", gpu_device, seed_param=[11, 12])
    assert [m for m, _ in calls] == ["prepare_condition", "generate_audio"]
    kw = calls[1][1]
    B, T = payload["src_latents"].shape[:2]
    cfg = _cfg()
    prep = out["prepare_condition"]
    passes0 = prep.passes
    with torch.inference_mode():
        enc, enc_mask, ctx = h.model.prepare_condition(**calls[0][1])    # service_generate_execute.py:123
        res = h.model.generate_audio(**kw)                               # service_generate_execute.py:194
    torch.cuda.synchronize()
    # one encoder pass serves both calls (the reference runs it twice: :123 and base:1820)
    assert prep.passes - passes0 == 1
    # conditioning = the oracle's AceStepConditionEncoder on the stub's weights
    cpu = {k: v.cpu() for k, v in kw.items() if isinstance(v, torch.Tensor)}
    with torch.no_grad():
        ref_enc, ref_mask = condenc_oracle.condition_encoder(
            {k: v.cpu() for k, v in h.model.CE.items()}, cfg, cpu["text_hidden_states"], cpu["text_attention_mask"],
            cpu["lyric_hidden_states"], cpu["lyric_attention_mask"], cpu["refer_audio_acoustic_hidden_states_packed"],
            cpu["refer_audio_order_mask"])
    assert torch.equal(enc_mask.cpu().bool(), ref_mask.cpu().bool())
    assert rel_l2(enc.float().cpu(), ref_enc.float().cpu()) <= 0.025
    assert cosine(enc.float().cpu(), ref_enc.float().cpu()) >= 0.999
    assert torch.equal(ctx, torch.cat([payload["src_latents"], payload["chunk_mask"]], -1))
    # generate_audio through install == the same backends built directly from the weights
    lat = res["target_latents"]
    assert lat.shape == (B, T, 64) and lat.dtype == torch.bfloat16 and torch.isfinite(lat.float()).all()
    assert set(res["time_costs"]) >= {"encoder_time_cost", "diffusion_time_cost", "diffusion_per_step_time_cost",
                                      "total_time_cost"}
    rt = DiTRuntime(cfg, gpu_device.index or 0, max_S=64, max_Bc=4, max_Lenc=64)
    rt.load(h.model.W)
    ce = ConditionEncoder(cfg, gpu_device.index or 0, max_batch=2)
    ce.load({"encoder." + k: v for k, v in h.model.CE.items()})
    be = AceStepDiTBackend(rt, h.model.null_condition_emb, prepare_condition=HipPrepareCondition(ce))
    with torch.inference_mode():
        direct = be.generate_audio(**kw)["target_latents"]
    torch.cuda.synchronize()
    assert torch.equal(direct, lat)
    rt.close()
    ce.close()
    # base variant: a `timesteps` kwarg is ignored, like the reference base (base:1812)
    assert out["dit"].accepts_timesteps is False

    # decode: handler.tiled_decode -> ONE untiled HIP decode of the batch
    # (generate_music_decode.py:123,164: transpose + cast to vae.dtype first)
    z = lat.transpose(1, 2).contiguous().to(h.vae.dtype)
    wav = h.tiled_decode(z)
    assert wav.shape == (B, 2, T * 1920) and wav.dtype == torch.float32
    for b in range(B):
        one = out["vae"].decode_tensor(z[b:b + 1].contiguous())
        torch.cuda.synchronize()
        assert torch.equal(wav[b:b + 1], one)
    assert torch.equal(h.vae.decode(z).sample, wav)                  # vae.decode seam too
    host = h.tiled_decode(z, offload_wav_to_cpu=True)
    assert host.device.type == "cpu" and torch.equal(host, wav.cpu())
    # offload_wav_to_cpu=None resolves through the handler's own policy (vae_decode.py:53-54)
    h.offload_policy = True
    assert h.tiled_decode(z).device.type == "cpu"
    h.offload_policy = False
    assert h.tiled_decode(z).is_cuda
    # encode seam: vae.encode(x).latent_dist.sample() (vae_encode.py:65)
    m = h.vae.encode(wav[:1].bfloat16()).latent_dist.mode()
    assert m.shape == (1, 64, T)
    # handler.tiled_encode (vae_encode.py:15-82) -> ONE untiled encode; the reference chunk loop
    # never runs (the stub's tiled_encode raises).  B = 2, 3-D and 2-D input, a sample count
    # that is not a multiple of hop, both offload settings; latent_dist.sample() semantics:
    # mean + std * eps, checked against the untiled encode with the same eps draw.
    vb = out["vae"]
    n = T * 1920 + 777
    g = torch.Generator(device=gpu_device).manual_seed(11)
    audio = (0.3 * torch.randn(2, 2, n, device=gpu_device, generator=g)).float()
    # placement (vae_encode.py:62-68): a source of <= chunk_size samples stays on the device even
    # with the reference default offload_latent_to_cpu=True; a longer one is offloaded
    torch.manual_seed(5)
    zs = h.tiled_encode(audio)
    assert zs.is_cuda and zs.shape == (2, 64, T) and zs.dtype == torch.bfloat16
    torch.manual_seed(5)
    ov = 1920                                                    # stride = chunk - 2·overlap > 0
    zc = h.tiled_encode(audio, chunk_size=n - 1, overlap=ov)    # "long" source: offloaded
    assert zc.device.type == "cpu" and torch.equal(zc, zs.cpu())
    torch.manual_seed(5)
    zg = h.tiled_encode(audio, chunk_size=n - 1, overlap=ov, offload_latent_to_cpu=False)
    assert zg.is_cuda and torch.equal(zg.cpu(), zc)
    torch.manual_seed(5)
    eps = torch.randn(2, 64, T, device=gpu_device, dtype=torch.bfloat16)
    direct = vb.encode_tensor(audio.bfloat16(), sample=True, eps=eps)
    torch.cuda.synchronize()
    assert torch.equal(zg, direct)
    mean = vb.encode_tensor(audio.bfloat16(), sample=False)
    assert not torch.equal(zg, mean)                             # a sample, not the mode
    z1 = h.tiled_encode(audio[1], offload_latent_to_cpu=False)  # [2, N] -> [64, T]
    assert z1.shape == (64, T)
    with pytest.raises(ValueError):                             # vae_encode.py:70-72: stride <= 0
        h.tiled_encode(audio, chunk_size=n - 1)                 # default overlap 2 s > chunk / 2
    torch.cuda.synchronize()


def test_install_lora_repack_vs_oracle(gpu_device, installed):
    """§8f row 3: after add_lora / set_lora_scale / unload_lora the handle holds the merged
    decoder weights; its forward equals the oracle on W + ΔW (and reverts exactly)."""
    h, out = installed
    rt = out["dit"].rt
    cfg = _cfg()
    g = torch.Generator().manual_seed(3)
    B, T, Le = 1, 50, 24
    xt = torch.randn(B, T, 64, generator=g).bfloat16()
    ctx = torch.randn(B, T, 128, generator=g).bfloat16()
    enc = torch.randn(B, Le, cfg.hidden_size, generator=g).bfloat16()
    t = torch.tensor([0.625], dtype=torch.float32, device=gpu_device)

    def hip():
        rt.set_condition(enc.to(gpu_device))
        o = rt.forward(xt.to(gpu_device), ctx.to(gpu_device), t).float().cpu()
        torch.cuda.synchronize()
        return o

    def oracle(W):
        Wb = {k: v.float().cpu().bfloat16() for k, v in W.items()}
        tb = torch.tensor([0.625], dtype=torch.bfloat16)
        with torch.no_grad():
            return dit_oracle.dit_forward(Wb, cfg, xt, tb, tb, enc, ctx).float()

    base = hip()
    ref_base = oracle(h.model.W)
    for scale in (1.0, 0.35):
        if scale == 1.0:
            h.add_lora("synthetic", scale=1.0)                   # wrapped by install -> re-pack
        else:
            h.set_lora_scale(scale)
        W = dict(h.model.W)
        for name in h.lora_targets:
            *parent, leaf = name.split(".")
            m = h.model.decoder
            for p in parent:
                m = m._modules[p]
            lo = m._modules[leaf]
            W[name + ".weight"] = (lo.base_layer.weight.float() + lo.get_delta_weight("default")).bfloat16()
        got, ref = hip(), oracle(W)
        assert rel_l2(got, ref) <= 0.025 and cosine(got, ref) >= 0.999, (scale, rel_l2(got, ref))
        # the adapters' effect (through gated residuals it is ~1 % of the output here) is
        # tracked: HIP's change equals the oracle's change
        assert rel_l2(got, base) > 0.004
        assert rel_l2(got - base, ref - ref_base) < 0.15, rel_l2(got - base, ref - ref_base)
    h.unload_lora()
    assert torch.equal(hip(), base)


def test_bench_two_ranks_on_one_gpu(gpu_device, tmp_path):
    """`bench.py --gpus 2` end to end on a one-GPU box (the path the driver's multi-GPU run takes:
    rank 0 conditions the batch of two songs and scatters it, both ranks run DiT + decode, the
    latents are gathered, the timing is max-over-ranks): ACEHIP_DIST_BACKEND=gloo lets both ranks
    share cuda:0 with host-staged collectives (RCCL refuses two ranks on one device).  Short songs
    so it fits the test budget; the JSON line must report both ranks' songs."""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ACEHIP_DIST_BACKEND="gloo", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--seconds", "10", "--no-cpu-baseline", "--no-config1"]
    p = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-2000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, p.stdout[-2000:]
    d = json.loads(lines[-1])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["parallelism"].endswith("x2"), d
