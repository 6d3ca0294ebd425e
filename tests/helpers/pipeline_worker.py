"""One rank of the SongParallelPipeline CPU test (started by acehip.distributed.launch_local,
gloo).  The DiT backend is a CPU stand-in with the same surface as AceStepDiTBackend
(``_condition``, ``_non_cover_condition``, ``generate_audio(**kw)`` honouring ``_noise`` /
``_non_cover`` / ``src_latents``): its "latents" are a fixed function of each song's own
encoder states, context, noise and sampler arguments, so a song computed on any rank must
equal the same song computed in the whole batch at once.  Rank 0 sends three requests (int
seed, seed list + cover noise, acs < 1 with B < world) and a stop, then two requests through a
pipeline with a stand-in VAE and gather_wav (B = 1 < world, B = 5); it checks every result
against the single-process batch computation and writes $ACEHIP_TEST_OUT/rank<r>.json."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]

import torch  # noqa: E402

from acehip import distributed as D  # noqa: E402
from acehip.dit import prepare_noise  # noqa: E402

LENC, D_MODEL, T = 6, 8, 10


class StubBackend:
    dtype = torch.float32
    device = torch.device("cpu")

    def __init__(self):
        self.calls = []

    def _condition(self, kw):
        text = kw["text_hidden_states"]
        enc = text[:, :LENC, :] * 2.0 + 1.0                       # "prepare_condition"
        ctx = torch.cat([kw["src_latents"], kw["chunk_masks"]], -1)
        return enc, None, ctx

    def _non_cover_condition(self, kw, ctx):
        return kw["non_cover_text_hidden_states"][:, :LENC, :] - 3.0, None, ctx * 0.5

    def generate_audio(self, **kw):
        enc, ctx = kw["encoder_hidden_states"], kw["context_latents"]
        B = ctx.shape[0]
        x = kw.get("_noise")
        if x is None:
            x = prepare_noise((B, ctx.shape[1], ctx.shape[2] // 2), self.device, self.dtype, kw.get("seed"))
        out = x * float(kw.get("infer_steps", 1)) + enc.mean(dim=(1, 2))[:, None, None] + ctx[..., :4].sum(-1, keepdim=True)
        if float(kw.get("cover_noise_strength", 0.0)) > 0:
            out = out + 0.25 * kw["src_latents"]
        if "_non_cover" in kw:
            enc_nc, ctx_nc = kw["_non_cover"]
            out = out + enc_nc.mean(dim=(1, 2))[:, None, None] + ctx_nc[..., :1]
        self.calls.append(B)
        return {"target_latents": out, "time_costs": {"total_time_cost": 0.0}}


class StubVAE:
    """decode_tensor(z [c, C, T]) → [c, 2, T·hop] fp32, a fixed function of z (CPU)."""

    class cfg:
        audio_channels, hop_length = 2, 3

    def decode_tensor(self, z):
        c, C, T = z.shape
        a = z.float().sum(1, keepdim=True)                            # [c, 1, T]
        return torch.cat([a, 2 * a], 1).repeat_interleave(3, dim=2)   # [c, 2, 3T]

    def postprocess_(self, wav, normalization_db=None):
        return wav


def request(B, seed, g, **extra):
    kw = dict(text_hidden_states=torch.randn(B, LENC + 2, D_MODEL, generator=g),
              src_latents=torch.randn(B, T, 4, generator=g), chunk_masks=torch.ones(B, T, 4),
              infer_steps=3, seed=seed, **extra)
    if extra.get("audio_cover_strength", 1.0) < 1.0:
        kw["non_cover_text_hidden_states"] = torch.randn(B, LENC + 2, D_MODEL, generator=g)
    return kw


def batch_reference(kw):
    """What the whole batch gives in one process (the reference's single-device batch)."""
    be = StubBackend()
    enc, _, ctx = be._condition(kw)
    if kw.get("audio_cover_strength", 1.0) < 1.0:
        enc_nc, _, ctx_nc = be._non_cover_condition(kw, ctx)
        kw = dict(kw, _non_cover=(enc_nc, ctx_nc))
    return be.generate_audio(encoder_hidden_states=enc, context_latents=ctx, **{k: v for k, v in kw.items()
                                                                             if k not in ("text_hidden_states",)})


def main():
    torch.set_num_threads(1)
    rank, world, _ = D.init(backend="gloo")
    be = StubBackend()
    pipe = D.SongParallelPipeline(be, None)
    rec = {"rank": rank, "world": world}
    if rank == 0:
        g = torch.Generator().manual_seed(5)
        reqs = [request(5, 1234, g),                                             # one generator, whole batch
                request(4, [3, None, 7, 11], g, cover_noise_strength=0.4),       # per-song seeds, src latents
                request(1, [9], g, audio_cover_strength=0.5)]                    # fewer songs than ranks
        ok = []
        for kw in reqs:
            res = pipe.generate(**kw)
            ref = batch_reference(kw)["target_latents"]
            if kw["seed"] is not None and isinstance(kw["seed"], list) and None in kw["seed"]:
                # the unseeded song's noise is random: compare the seeded rows only
                rows = [i for i, s in enumerate(kw["seed"]) if s is not None]
                ok.append(bool(torch.equal(res["target_latents"][rows], ref[rows])))
            else:
                ok.append(bool(torch.equal(res["target_latents"], ref)))
        pipe.stop()
        # with a VAE and gather_wav: audio gathered in batch order, also when B < world (ranks
        # without songs still join the gather)
        pipe2 = D.SongParallelPipeline(be, StubVAE(), gather_wav=True, normalization_db=None)
        for B in (1, 5):
            kw = request(B, 77 + B, g)
            res = pipe2.generate(**kw)
            ref = batch_reference(kw)["target_latents"]
            want = StubVAE().decode_tensor(ref.transpose(1, 2))
            ok.append(bool(torch.equal(res["wav"], want)) and tuple(res["wav"].shape) == (B, 2, 3 * T))
        pipe2.stop()
        rec["ok"] = ok
    else:
        pipe.serve()
        D.SongParallelPipeline(be, StubVAE(), gather_wav=True, normalization_db=None).serve()
    rec["calls"] = be.calls
    D.barrier()
    with open(os.path.join(os.environ["ACEHIP_TEST_OUT"], f"rank{rank}.json"), "w") as f:
        json.dump(rec, f)
    D.destroy()


if __name__ == "__main__":
    main()
