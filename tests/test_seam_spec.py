"""CPU checks of the recorded reference seam (tests/golden/seam_calls.json, written by
tools/record_seam.py from service_generate_execute.py:62-196) and of the one-pass-per-request
conditioning memo that install() binds to it."""
import inspect

import torch

from seam_spec import build_calls, load_spec

from acehip.condition import HipPrepareCondition
from acehip.distributed import _CONDITION_KW, _SAMPLER_KW

# reference generate_audio parameters: base / sft / turbo signatures
# (base:1783-1813, sft adds timesteps, turbo:1780-1806 adds fix_nfe)
REF_GENERATE_AUDIO = {
    "text_hidden_states", "text_attention_mask", "lyric_hidden_states", "lyric_attention_mask",
    "refer_audio_acoustic_hidden_states_packed", "refer_audio_order_mask", "src_latents", "chunk_masks",
    "is_covers", "silence_latent", "attention_mask", "seed", "fix_nfe", "infer_method", "use_cache",
    "infer_steps", "diffusion_guidance_sale", "audio_cover_strength", "non_cover_text_hidden_states",
    "non_cover_text_attention_mask", "cfg_interval_start", "cfg_interval_end", "precomputed_lm_hints_25Hz",
    "audio_codes", "use_progress_bar", "use_adg", "shift", "timesteps", "cover_noise_strength"}


def test_spec_shape():
    spec = load_spec()
    assert set(spec["scenarios"]) == {"base_seed_list", "custom_timesteps", "random_seed"}
    for name, sc in spec["scenarios"].items():
        methods = [c["method"] for c in sc["calls"]]
        assert methods == ["prepare_condition", "generate_audio"], (name, methods)
        gen = {e["name"]: e for e in sc["calls"][1]["kwargs"]}
        assert set(gen) <= REF_GENERATE_AUDIO
        # every generate_audio keyword is either conditioning (rank 0 turns it into tensors) or a
        # sampler keyword the song-parallel pipeline forwards to every rank
        assert set(gen) <= set(_CONDITION_KW) | set(_SAMPLER_KW), set(gen) - set(_CONDITION_KW) - set(_SAMPLER_KW)
        assert gen["seed"]["value"] == "seed_param"
        assert ("timesteps" in gen) == (name == "custom_timesteps")
        if "timesteps" in gen:
            assert gen["timesteps"]["dtype"] == "float32" and gen["timesteps"]["source"] == "fresh"
        prep = {e["name"]: e for e in sc["calls"][0]["kwargs"]}
        assert set(prep) <= set(inspect.signature(HipPrepareCondition.__call__).parameters)
        # the handler's call and generate_audio's condition the SAME payload tensors
        for k in HipPrepareCondition._MEMO_KEYS:
            if k in prep and prep[k]["kind"] == "tensor" and k in gen:
                assert prep[k]["source"] == gen[k]["source"], k
        assert prep["hidden_states"]["source"] == gen["src_latents"]["source"] == "payload:src_latents"
        assert prep["attention_mask"]["source"] == "fresh" and prep["attention_mask"]["values"]["all_ones"]


def test_build_calls_shares_objects():
    payload, silence, calls = build_calls("custom_timesteps", torch.device("cpu"), seed_param=[5, 6])
    prep, gen = calls[0][1], calls[1][1]
    assert prep["text_hidden_states"] is gen["text_hidden_states"] is payload["text_hidden_states"]
    assert prep["hidden_states"] is gen["src_latents"] is payload["src_latents"]
    assert gen["silence_latent"] is silence and gen["seed"] == [5, 6]
    assert torch.equal(gen["timesteps"], torch.tensor([1.0, 0.75, 0.5, 0.25]))


class _FakeEncoder:
    def __init__(self):
        self.calls = 0

    def __call__(self, th, tm, lh, lm, ra, ro):
        self.calls += 1
        B = th.shape[0]
        return torch.full((B, 3, 4), float(self.calls)), torch.ones(B, 3)


def test_memo_one_pass_per_request():
    _, _, calls = build_calls("base_seed_list", torch.device("cpu"), seed_param=[1, 2])
    prep_kw = calls[0][1]
    enc = _FakeEncoder()
    hp = HipPrepareCondition(enc)
    gen_side = dict(prep_kw, attention_mask=torch.ones_like(prep_kw["attention_mask"]))  # a new ones mask
    a = hp.record(**prep_kw)
    b = hp.consume(**gen_side)
    assert enc.calls == 1 and hp.passes == 1 and b is a
    # single use: a second consume (e.g. the next request on the same tensors) recomputes
    hp.consume(**gen_side)
    assert enc.calls == 2
    # a different tensor object recomputes
    hp.record(**prep_kw)
    other = dict(gen_side, lyric_hidden_states=prep_kw["lyric_hidden_states"].clone())
    hp.consume(**other)
    assert enc.calls == 4
    # an in-place change between the two calls (version bump) recomputes
    hp.record(**prep_kw)
    prep_kw["src_latents"].add_(0)
    hp.consume(**gen_side)
    assert enc.calls == 6
    # a direct call never stores: consume after __call__ recomputes (bench.py's path)
    hp(**prep_kw)
    hp.consume(**gen_side)
    assert enc.calls == 8
