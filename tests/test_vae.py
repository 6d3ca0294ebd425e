"""Oobleck VAE: oracle structure checks (CPU) and HIP decode/encode parity vs
the fp32 CPU oracle (GPU).  VAE parity is UNPINNED against the reference
(diffusers AutoencoderOobleck is absent; see oracle/vae_oracle.py)."""
import os

import pytest
import torch

from conftest import cosine, rel_l2

from acehip.config import VAEConfig
from acehip.weights import synth_vae_weights, vae_weight_shapes
from oracle import vae_oracle


def test_vae_hop_and_shapes():
    cfg = VAEConfig()
    assert cfg.hop_length == 1920                      # conditioning_masks.py:42-43
    assert cfg.decoder_block_channels()[0] == (2048, 1024, 10)
    s = vae_weight_shapes(cfg)
    assert s["decoder.conv1.weight_v"] == (2048, 64, 7)
    assert s["decoder.block.0.conv_t1.weight_v"] == (2048, 1024, 20)   # ConvT: [in, out, k]
    assert s["decoder.block.0.conv_t1.weight_g"] == (2048, 1, 1)       # norm over dim 0 = input ch
    assert s["encoder.conv2.weight_v"] == (128, 2048, 3)


def test_weight_norm_fusion_matches_torch():
    v = torch.randn(6, 4, 3)
    g = torch.rand(6, 1, 1) + 0.5
    conv = torch.nn.utils.parametrizations.weight_norm(torch.nn.Conv1d(4, 6, 3), dim=0)
    with torch.no_grad():
        conv.parametrizations.weight.original0.copy_(g)
        conv.parametrizations.weight.original1.copy_(v)
    assert torch.allclose(vae_oracle.fuse_weight_norm(g, v), conv.weight, atol=1e-6)


def test_weight_norm_fusion_matches_reference_converter():
    """The oracle's weight-norm fusion against the reference's own converter
    (acestep/models/mlx/vae_convert.py:19-34 `_fuse_weight_norm`, numpy; fixture recorded by
    tools/record_vae_seam.py) on Conv1d and ConvTranspose1d shapes of the decoder: the converter
    adds 1e-9 to the norm (torch weight_norm, the GPU reference's path, does not), which is below
    fp32 resolution at these norms."""
    from conftest import load_golden
    t = load_golden("vae_weight_norm")
    names = sorted({k.rsplit(".", 1)[0] for k in t})
    assert len(names) == 6
    for n in names:
        got = vae_oracle.fuse_weight_norm(t[n + ".weight_g"], t[n + ".weight_v"])
        assert got.shape == t[n + ".fused"].shape
        assert torch.allclose(got, t[n + ".fused"], rtol=2e-6, atol=1e-9), n


def test_reference_tiled_decode_fixture():
    """The reference's own tiled decode (vae_decode_chunks.py:13-166), recorded with an indexing
    stand-in VAE (tools/record_vae_seam.py): for every (T, chunk, overlap 64, GPU / offload path) the
    stitched output is exactly the untiled sample sequence — the property acehip's untiled decode
    relies on (tests/test_gpu_long.py replays the same windows through the HIP decoder)."""
    import json
    from conftest import GOLDEN
    d = json.load(open(os.path.join(GOLDEN, "vae_seam.json")))
    hop = d["hop"]
    assert len(d["cases"]) == 40
    for c in d["cases"]:
        assert c["stitched_is_untiled"], (c["T"], c["chunk"], c["offload_wav_to_cpu"])
        assert sum(k1 - k0 for k0, k1 in c["keep"]) == c["T"] * hop
        pos = 0
        for (w0, w1), (k0, k1) in zip(c["windows"], c["keep"]):
            assert w0 * hop + k0 == pos and 0 <= k0 < k1 <= (w1 - w0) * hop
            pos += k1 - k0
    for c in d["encode_cases"]:
        assert c["stitched_is_untiled"], (c["T"], c["chunk"], c["offload_latent_to_cpu"])
        assert sum(k1 - k0 for k0, k1 in c["keep"]) == c["T"]
    # 240 s at the reference's largest chunk: 16 windows, 1.32x the useful frames decoded
    c = next(c for c in d["cases"] if c["T"] == 6000 and c["chunk"] == 512 and not c["offload_wav_to_cpu"])
    assert len(c["windows"]) == 16 and c["decoded_frames"] == 7920


def test_tiny_decoder_runs_on_cpu():
    cfg = VAEConfig.tiny()
    W = synth_vae_weights(cfg, seed=3, mode="parity", with_encoder=True)
    z = torch.randn(1, 64, 3)
    wav = vae_oracle.decode(W, cfg, z)
    assert wav.shape == (1, 2, 3 * 1920) and torch.isfinite(wav).all()
    lat = vae_oracle.encode_sample(W, cfg, wav)
    assert lat.shape == (1, 64, 3)


def _hip_vae(cfg, W, dev, max_T, with_encoder=True):
    from acehip.vae import OobleckBackend
    be = OobleckBackend(cfg, dev.index or 0, max_T=max_T, with_encoder=with_encoder)
    be.load({k: v.to(dev) for k, v in W.items()})
    return be


@pytest.mark.gpu
# tiny T = 7: every stage is C = 128 (the ru8 residual unit) and the last stage's L = 13440 is not a
# multiple of its 256-row tile, so the last window reaches ~300 rows past L into the back pad
@pytest.mark.parametrize("cfg_name,T", [("tiny", 6), ("tiny", 7), ("full", 8)])
def test_vae_decode_parity(gpu_device, cfg_name, T):
    cfg = VAEConfig.tiny() if cfg_name == "tiny" else VAEConfig()
    W = synth_vae_weights(cfg, seed=5, mode="parity", with_encoder=True)
    z = torch.randn(2, 64, T, generator=torch.Generator().manual_seed(T)).bfloat16()
    with torch.no_grad():
        ref = vae_oracle.decode(W, cfg, z.float())
        # calibration: the same restatement run in bf16 (what diffusers does on
        # the GPU) vs fp32 — 7.8 % on the full config at T=8
        spread = rel_l2(vae_oracle.decode({k: v.bfloat16() for k, v in W.items()}, cfg, z).float(), ref)
    be = _hip_vae(cfg, W, gpu_device, max_T=16)
    out = be.decode(z.to(gpu_device)).sample
    torch.cuda.synchronize()
    out = out.cpu()
    assert out.shape == ref.shape
    # bf16 activations through ~35 convolutions: within the bf16 spread (+1 %)
    assert rel_l2(out, ref) <= max(0.03, spread + 0.01), (rel_l2(out, ref), spread)
    assert cosine(out, ref) > 0.995
    be.close()


def test_oracle_encode_ragged_length():
    """AutoencoderOobleck's strided convs (k = 2s, pad ceil(s/2)) floor the length at every
    stage: N samples → floor(N / hop) latent frames, and the tail samples past
    hop·floor(N / hop) still reach the last frame through the right halo."""
    cfg = VAEConfig.tiny()
    W = synth_vae_weights(cfg, seed=3, mode="parity", with_encoder=True)
    g = torch.Generator().manual_seed(2)
    wav = 0.3 * torch.randn(1, 2, 3 * 1920 + 1500, generator=g)
    with torch.no_grad():
        z = vae_oracle.encode_sample(W, cfg, wav)
        zt = vae_oracle.encode_sample(W, cfg, wav[:, :, :3 * 1920])
    assert z.shape == (1, 64, 3)
    assert not torch.allclose(z[:, :, -1], zt[:, :, -1])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg_name,extra,B", [("tiny", 0, 1), ("full", 0, 1), ("tiny", 777, 2),
                                              ("full", 1919, 2)])
def test_vae_encode_parity(gpu_device, cfg_name, extra, B):
    """Encode parity vs the fp32 oracle, including sample counts that are not a multiple of
    hop (the handler's tiled_encode seam takes raw source audio)."""
    cfg = VAEConfig.tiny() if cfg_name == "tiny" else VAEConfig()
    W = synth_vae_weights(cfg, seed=6, mode="parity", with_encoder=True)
    g = torch.Generator().manual_seed(1)
    T = 3
    wav = (0.3 * torch.randn(B, 2, T * 1920 + extra, generator=g)).bfloat16()
    eps = torch.randn(B, 64, T, generator=g).bfloat16()
    with torch.no_grad():
        ref_mean = vae_oracle.encode_sample(W, cfg, wav.float())
        ref_s = vae_oracle.encode_sample(W, cfg, wav.float(), eps.float())
    be = _hip_vae(cfg, W, gpu_device, max_T=8)
    mean = be.encode_tensor(wav.to(gpu_device), sample=False).float().cpu()
    smp = be.encode_tensor(wav.to(gpu_device), eps=eps).float().cpu()
    assert mean.shape == ref_mean.shape == (B, 64, T)
    assert rel_l2(mean, ref_mean) < 0.03, rel_l2(mean, ref_mean)
    assert rel_l2(smp, ref_s) < 0.03
    be.close()


@pytest.mark.gpu
def test_vae_two_handles_alternate(gpu_device):
    """Launch state is per handle (each handle's own zero page goes into the conv
    arguments): two handles with different weights, decoding alternately and from two
    host threads, give exactly what each gives alone."""
    import threading
    cfg = VAEConfig.tiny()
    bes = [_hip_vae(cfg, synth_vae_weights(cfg, seed=s, mode="parity", with_encoder=True), gpu_device, 8)
           for s in (21, 22)]
    g = torch.Generator().manual_seed(9)
    zs = [torch.randn(1, 64, 6, generator=g).bfloat16().to(gpu_device) for _ in range(2)]
    alone = []
    for be, z in zip(bes, zs):
        alone.append(be.decode_tensor(z))
        torch.cuda.synchronize()
    for _ in range(3):
        for i in (1, 0):
            o = bes[i].decode_tensor(zs[i])
            torch.cuda.synchronize()
            assert torch.equal(o, alone[i])
    res = [None, None]

    def run(i):
        s = torch.cuda.Stream(device=gpu_device)
        with torch.cuda.stream(s):
            outs = [bes[i].decode_tensor(zs[i]) for _ in range(4)]
        s.synchronize()
        res[i] = all(torch.equal(o, alone[i]) for o in outs)
    th = [threading.Thread(target=run, args=(i,)) for i in (0, 1)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert res == [True, True]
    for be in bes:
        be.close()


@pytest.mark.gpu
def test_decode_guard_vs_reference_function(gpu_device):
    """The peak guard against the reference's own `_decode_generate_music_pred_latents`
    (generate_music_decode.py:98-201), recorded by tools/record_vae_seam.py with a stand-in bf16
    VAE: songs with a peak above 1, below 1, near silence and exactly 1 — bit-exact, through both
    product entry points (the guard alone and the guard + normalize pass with normalization off)."""
    from conftest import load_golden
    from acehip.vae import OobleckBackend
    t = load_golden("decode_guard")
    x = t["wav_bf16"].float().to(gpu_device).contiguous()      # the handler's .float() (:188-189)
    a = x.clone()
    OobleckBackend.peak_normalize_(a)
    b = x.clone()
    OobleckBackend.postprocess_(b, normalization_db=None)
    torch.cuda.synchronize()
    assert torch.equal(a.cpu(), t["pred_wavs"])
    assert torch.equal(b.cpu(), t["pred_wavs"])


@pytest.mark.gpu
def test_wav_peak_normalize(gpu_device):
    """generate_music_decode.py:190-192 output guard, bit-exact vs the torch formula."""
    from acehip.vae import OobleckBackend
    from acehip.config import VAEConfig
    be = OobleckBackend(VAEConfig.tiny(), 0, max_T=8, with_encoder=False)
    g = torch.Generator().manual_seed(4)
    wav = torch.randn(3, 2, 3840 * 5, generator=g)
    wav[0] *= 0.2            # peak < 1: untouched
    wav[1] *= 2.5            # peak > 1: divided
    wav[2, 1, 77] = -7.0     # negative extreme sets the peak
    ref = wav.clone()
    peak = ref.abs().amax(dim=[1, 2], keepdim=True)
    if torch.any(peak > 1.0):
        ref = ref / peak.clamp(min=1.0)
    out = be.peak_normalize_(wav.to(gpu_device).contiguous())
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ref)
    be.close()


@pytest.mark.gpu
@pytest.mark.parametrize("db", [-1.0, -3.0, 0.0, None])
def test_wav_postprocess_guard_plus_normalize(gpu_device, db):
    """§8f row 4: decode guard + normalize_audio fused in one HIP pass pair, bit-exact
    against the reference's two steps (oracle/audio_oracle.py restates them)."""
    from acehip.vae import OobleckBackend
    from acehip.config import VAEConfig
    from oracle import audio_oracle
    be = OobleckBackend(VAEConfig.tiny(), 0, max_T=8, with_encoder=False)
    g = torch.Generator().manual_seed(5)
    wav = torch.randn(5, 2, 3840 * 7, generator=g)
    wav[0] *= 0.2            # peak < 1: only normalized
    wav[1] *= 2.5            # peak > 1: guard, then normalized
    wav[2, 1, 77] = -7.0     # negative extreme sets the peak
    wav[3] *= 1e-8           # near-silence: normalize_audio returns it unchanged
    wav[4] = 0.0             # silence
    ref = audio_oracle.decode_guard(wav.clone())
    if db is not None:
        ref = torch.stack([audio_oracle.normalize_audio(ref[b], db) for b in range(ref.shape[0])])
    out = be.postprocess_(wav.to(gpu_device).contiguous(), normalization_db=db)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ref)
    be.close()


def test_normalize_audio_oracle_vs_reference_function():
    """oracle.audio_oracle.normalize_audio against the reference's own normalize_audio
    (audio_utils.py:24-62), recorded by tools/record_vae_seam.py: bit-exact."""
    from conftest import load_golden
    from oracle import audio_oracle
    t = load_golden("normalize_audio")
    for i in range(5):
        out = audio_oracle.normalize_audio(t[f"case{i}.in"], float(t[f"case{i}.db"][0]))
        assert torch.equal(out, t[f"case{i}.out"]), i


@pytest.mark.gpu
def test_hip_normalize_audio_vs_reference_fixture(gpu_device):
    """integration.hip_normalize_audio against the reference function's recorded outputs."""
    from conftest import load_golden
    from acehip.integration import hip_normalize_audio
    t = load_golden("normalize_audio")
    for i in range(5):
        out = hip_normalize_audio(t[f"case{i}.in"].to(gpu_device), float(t[f"case{i}.db"][0]))
        torch.cuda.synchronize()
        assert torch.equal(out.cpu(), t[f"case{i}.out"]), i


@pytest.mark.gpu
@pytest.mark.parametrize("scale,db", [(3.0, -1.0), (0.3, -1.0), (1e-8, -1.0), (0.7, -6.0)])
def test_hip_normalize_audio_matches_reference(gpu_device, scale, db):
    """integration.hip_normalize_audio (normalize_audio for device tensors, no guard)."""
    from acehip.integration import hip_normalize_audio
    from oracle import audio_oracle
    a = torch.randn(2, 48000, generator=torch.Generator().manual_seed(2)) * scale
    ref = audio_oracle.normalize_audio(a, db)
    out = hip_normalize_audio(a.to(gpu_device), db)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ref)


def _oracle_stage(W, cfg, j, xs):
    """Decoder stage j of the fp32 oracle (vae_model.py:119-142, 190-230) from the snaked input
    xs [1, C, L] (channels-first): stage 0 = conv1 + block 0's snake1 applied to z; stage
    1 + j = block j (ConvT → 3 residual units) + the next Snake; the last = conv2."""
    import math
    import torch.nn.functional as F
    blocks = cfg.decoder_block_channels()
    if j == 0:
        x = F.conv1d(xs, vae_oracle._w(W, "decoder.conv1"), W["decoder.conv1.bias"], padding=3)
        return vae_oracle._snake(W, "decoder.block.0.snake1", x)
    if j == len(blocks) + 1:
        return F.conv1d(xs, vae_oracle._w(W, "decoder.conv2"), None, padding=3)
    b = j - 1
    p, s = f"decoder.block.{b}", blocks[b][2]
    x = F.conv_transpose1d(xs, vae_oracle._w(W, p + ".conv_t1"), W[p + ".conv_t1.bias"], stride=s,
                           padding=math.ceil(s / 2))
    for n, d in ((1, 1), (2, 3), (3, 9)):
        x = vae_oracle._res_unit(W, f"{p}.res_unit{n}", x, d)
    nxt = f"decoder.block.{b + 1}.snake1" if b + 1 < len(blocks) else "decoder.snake1"
    return vae_oracle._snake(W, nxt, x)


VAE_STAGE_TOL = 0.025   # measured ≤ 1.7 % (block 0, C = 1024)


@pytest.mark.gpu
@pytest.mark.parametrize("T", [8, 150])
def test_vae_decode_stagewise_parity(gpu_device, T):
    """Block-level parity of the full-width decoder (acehip_vae_decode_blocks): each stage of the
    HIP decoder — conv1, the five blocks (ConvT + three residual units + the next Snake), conv2 —
    against the fp32 oracle applied to the HIP path's OWN bf16 input of that stage, so a stage's
    error is not buried under the ~5 % rounding spread that 35 bf16 convolutions of this
    random-weight decoder accumulate end to end (oracle bf16-storage vs fp32: 5.1 % at 240 s,
    tools/vae_parity_probe.py).  The last stage is the product's own decode output."""
    from acehip import _ffi as ff
    cfg = VAEConfig()
    W = synth_vae_weights(cfg, seed=5, mode="parity", with_encoder=False)
    Wd = {k: v.to(gpu_device) for k, v in W.items()}
    be = _hip_vae(cfg, W, gpu_device, max_T=T, with_encoder=False)
    z = torch.randn(1, 64, T, generator=torch.Generator().manual_seed(T)).bfloat16().to(gpu_device)
    blocks = cfg.decoder_block_channels()
    acts, L, C = [], T, blocks[0][0]
    for j in range(len(blocks) + 1):
        if j:
            L, C = L * blocks[j - 1][2], blocks[j - 1][1]
        a = torch.empty(L, C, device=gpu_device, dtype=torch.bfloat16)
        ff.check(ff.lib().acehip_vae_decode_blocks(be.h, ff.ptr(z), T, j, ff.ptr(a), ff.stream_ptr()), "decode_blocks")
        acts.append(a.t().unsqueeze(0).float())             # [1, C, L]
    wav = be.decode(z).sample.float()
    torch.cuda.synchronize()
    outs = acts + [wav]
    errs = []
    with torch.no_grad():
        for j in range(len(outs)):
            src = z.float() if j == 0 else acts[j - 1]
            ref = _oracle_stage(Wd, cfg, j, src)
            errs.append(rel_l2(outs[j].cpu(), ref.cpu()))
    print(f"VAE stagewise T={T}: " + " ".join(f"{e:.2e}" for e in errs))
    assert all(e <= VAE_STAGE_TOL for e in errs), errs
    be.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg_name,T", [("tiny", 7), ("full", 150), ("full", 6000)])
def test_vae_snake_in_blocks(gpu_device, monkeypatch, cfg_name, T):
    """C = 128 decoder blocks on the snake-in path (ACEHIP_VAE_SNAKE_IN=1, default): the residual
    units stage raw x and apply their first Snake while staging (no x_s tensors; ConvT writes raw
    x only, units 1-2 raw x' only, to a second buffer) — the same values as the x_s path
    (ACEHIP_VAE_SNAKE_IN=0), which computes the same Snake in the producer's epilogue."""
    from conftest import set_knob
    cfg = VAEConfig.tiny() if cfg_name == "tiny" else VAEConfig()
    W = synth_vae_weights(cfg, seed=9, mode="parity", with_encoder=False)
    be = _hip_vae(cfg, W, gpu_device, max_T=T, with_encoder=False)
    z = torch.randn(1, 64, T, generator=torch.Generator().manual_seed(T + 3)).bfloat16().to(gpu_device)
    outs = {}
    for v in ("0", "1"):
        set_knob(monkeypatch, "ACEHIP_VAE_SNAKE_IN", v)
        outs[v] = be.decode(z).sample.clone()
        torch.cuda.synchronize()
    be.close()
    a, b = outs["0"].float().cpu(), outs["1"].float().cpu()
    assert torch.isfinite(b).all()
    d = (a - b).abs().max().item()
    print(f"snake-in vs x_s path {cfg_name} T={T}: max |diff| {d:.3e}, rel-L2 {rel_l2(b, a):.3e}")
    assert rel_l2(b, a) < 1e-3, (d, rel_l2(b, a))
