"""The fp32 parity mode (rel-L2 <= 1e-4 vs the
reference's fp32 forward): a DiT handle created with ``fp32=1`` runs
``AceStepDiTModel.forward`` in fp32 end to end (f32.hip: exact-fp32 MFMA GEMMs
and attention); checked against the reference's own fp32 outputs
(``tests/golden/dit_fwd_*_float32``, made by tools/make_golden.py) — tiny configs
(even / odd T, band ±8 with S > 2W), full width at T = 64 and T = 641 (S = 321 > 257:
the ±128 band pinned at full width)."""
import pytest
import torch

from conftest import cosine, golden_manifest, load_golden, rel_l2

from acehip.config import DiTConfig
from acehip.weights import synth_dit_weights
from oracle import dit_oracle

pytestmark = pytest.mark.gpu

TOL_FP32 = 1e-4


@pytest.mark.parametrize("name", ["tiny_float32", "tiny_odd_float32", "full2_float32", "full2_long_float32"])
def test_fp32_forward_vs_reference_golden(gpu_device, name):
    from acehip.dit import DiTRuntime
    meta = golden_manifest()["forward"][name]
    cfg = DiTConfig(**meta["cfg"])
    g = load_golden("dit_fwd_" + name)
    W = synth_dit_weights(cfg, seed=meta["seed"], mode="parity")          # fp32, checksum-pinned
    rt = DiTRuntime(cfg, gpu_device.index or 0, max_S=max(64, (meta["T"] + 1) // 2),
                    max_Bc=meta["B"], max_Lenc=max(32, meta["Lenc"]), dtype=torch.float32)
    rt.load({k: v.to(gpu_device) for k, v in W.items()})
    rt.set_condition(g["enc"].to(gpu_device))
    out = rt.forward(g["xt"].to(gpu_device).contiguous(), g["ctx"].to(gpu_device).contiguous(),
                     g["t"].to(gpu_device), g["t_r"].to(gpu_device))
    torch.cuda.synchronize()
    out = out.cpu()
    assert out.dtype == torch.float32
    r = rel_l2(out, g["vt"])
    assert r <= TOL_FP32, (name, r)
    rt.close()


def test_fp32_cfg_rows_vs_oracle(gpu_device):
    """Bx = 1 < Bc = 2 (CFG reads xt row b % Bx), null rows present (set_uniform_rows is a
    no-op in the parity mode: every row computed in full), odd T, Lenc not a multiple of
    anything — vs the fp32 oracle."""
    from acehip.dit import DiTRuntime
    cfg = DiTConfig.tiny(layers=3, window=16)
    W = synth_dit_weights(cfg, seed=8, mode="parity")
    gen = torch.Generator().manual_seed(4)
    T, Lenc = 301, 45
    xt = torch.randn(1, T, 64, generator=gen)
    ctx = torch.randn(1, T, 128, generator=gen)
    enc = torch.randn(1, Lenc, cfg.hidden_size, generator=gen)
    null = torch.randn(1, 1, cfg.hidden_size, generator=gen)
    enc2 = torch.cat([enc, null.expand_as(enc)])
    t = torch.tensor([0.3125])
    with torch.no_grad():
        ref = dit_oracle.dit_forward(W, cfg, torch.cat([xt, xt]), t.expand(2), t.expand(2), enc2,
                                     torch.cat([ctx, ctx]))
    rt = DiTRuntime(cfg, gpu_device.index or 0, max_S=160, max_Bc=2, max_Lenc=64, dtype=torch.float32)
    rt.load({k: v.to(gpu_device) for k, v in W.items()})
    rt.set_condition(enc2.to(gpu_device))
    rt.set_uniform_rows(1)
    out = rt.forward(xt.to(gpu_device), ctx.to(gpu_device), t.to(gpu_device)).cpu()
    torch.cuda.synchronize()
    assert rel_l2(out, ref) <= TOL_FP32 and cosine(out, ref) > 0.9999999
    # the handle refuses bf16 inputs: the ABI's dtype argument must match the handle
    with pytest.raises(AssertionError):
        rt.forward(xt.bfloat16().to(gpu_device), ctx.bfloat16().to(gpu_device), t.to(gpu_device))
    rt.close()


def test_fp32_generate_audio_per_step(gpu_device):
    """generate_audio in the fp32 parity mode end to end (fp32 DiT handle + the fp32
    instantiation of the fused APG/Euler kernel): every step's DiT output vs the fp32
    oracle fed the same x_t (<= 1e-4), and the trajectory vs the oracle sampler driven
    by the HIP outputs (fp32 APG: fp64 projections, fp32 elsewhere)."""
    from acehip.dit import AceStepDiTBackend, DiTRuntime
    from oracle import sampler_oracle
    cfg = DiTConfig.tiny(layers=2, window=8)
    W = synth_dit_weights(cfg, seed=9, mode="parity")
    null = torch.randn(1, 1, cfg.hidden_size, generator=torch.Generator().manual_seed(1))
    rt = DiTRuntime(cfg, gpu_device.index or 0, max_S=64, max_Bc=4, max_Lenc=32, dtype=torch.float32)
    rt.load({k: v.to(gpu_device) for k, v in W.items()})
    be = AceStepDiTBackend(rt, null, dtype=torch.float32)
    g = torch.Generator().manual_seed(0)
    B, T, Lenc = 2, 60, 24
    enc = torch.randn(B, Lenc, cfg.hidden_size, generator=g)
    ctx = torch.randn(B, T, 128, generator=g)
    seen = []
    orig = rt.forward

    def spy(xt, c, t, t_r=None, out=None):
        vt = orig(xt, c, t, t_r, out)
        seen.append((xt.clone(), t.clone(), vt.clone()))
        return vt
    rt.forward = spy
    res = be.generate_audio(encoder_hidden_states=enc.to(gpu_device), context_latents=ctx.to(gpu_device),
                            infer_steps=4, diffusion_guidance_sale=7.0, shift=3.0, seed=[0, 1])
    torch.cuda.synchronize()
    out = res["target_latents"].cpu()
    assert out.dtype == torch.float32 and len(seen) == 4
    enc2 = torch.cat([enc, null.expand_as(enc)])
    kv = dit_oracle.cross_kv(W, cfg, enc2)
    for xt, t, vt in seen:
        tv = t.cpu().expand(2 * B)
        with torch.no_grad():
            ref = dit_oracle.dit_forward(W, cfg, torch.cat([xt, xt]).cpu(), tv, tv, enc2, torch.cat([ctx, ctx]),
                                         kv_cache=kv)
        assert rel_l2(vt.cpu(), ref) <= TOL_FP32, rel_l2(vt.cpu(), ref)
    # the sampler arithmetic around the DiT: the oracle's base loop replaying the HIP outputs
    it = iter([v.cpu() for _, _, v in seen])
    ref_x = sampler_oracle.generate_base(lambda x, tv: next(it), seen[0][0].cpu(), 4, guidance=7.0, shift=3.0)
    assert rel_l2(out, ref_x) <= 1e-5
    rt.close()
