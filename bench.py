#!/usr/bin/env python3
"""bench.py — seconds/song for ACE-Step 1.5 text2music on the HIP path.

Workload (BASELINE.json configs[1]): a 240 s song
(T = 6000 latent frames, S = 3000 tokens), base/sft schedule with 27 steps,
shift 3, CFG guidance 7 (DiT batch Bc = 2) with APG, ODE/Euler, bf16, the
full-size 24-layer DiT (random init, synthetic conditioning enc [1,641,2048],
context [silence N(0,1) | ones]) followed by the full Oobleck VAE decode to
48 kHz stereo.  One bench "step" = one song through the whole hot path
(27 DiT forwards + 27 fused APG/Euler steps + VAE decode).

Multi-GPU (``--gpus N``): one song per GPU per step (song-parallel, SURVEY
§8e), one process per GPU.  Under a launcher (torchrun sets WORLD_SIZE) the
ranks come from the environment and must equal N; started plainly with N > 1,
bench.py spawns the N ranks itself (``acehip.distributed.launch_local``, before
anything touches the GPU).  Rank 0 conditions each step's batch once and scatters each
rank its song (acehip.distributed.SongParallelPipeline) over RCCL, no
collective inside the timed work; value = max-over-ranks time ÷ all songs.
``--dry-run`` runs the same harness on CPU ranks over gloo with a stand-in song
(the multi-rank CPU test drives it).

Prints ONE JSON line on rank 0.  ``roofline`` is the dominant kernel (the
SwiGLU gate/up GEMM, 2·M·N·K algorithmic FLOPs per launch) timed with HIP
events around every launch inside the timed region; ``cpu_baseline`` is the
CPU oracle (PyTorch fp32) timed on this host for one full-size CFG DiT step +
a 64-frame VAE window, extrapolated to the song.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]

import torch  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--seconds", type=float, default=240.0)
    p.add_argument("--infer-steps", type=int, default=27)
    p.add_argument("--guidance", type=float, default=7.0)
    p.add_argument("--shift", type=float, default=3.0)
    p.add_argument("--lenc", type=int, default=641)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-vae", action="store_true")
    p.add_argument("--graph", action="store_true",
                   help="replay each forward's layer stack as a captured HIP graph (measured neutral; off by default)")
    p.add_argument("--no-condition", action="store_true",
                   help="feed synthetic encoder states directly (skip the HIP condition encoders)")
    p.add_argument("--lyric-len", type=int, default=512)
    p.add_argument("--turbo", action="store_true",
                   help="turbo sampler (table schedule, no CFG; SURVEY config 1 shape: --seconds 10 --infer-steps 8)")
    p.add_argument("--no-overlap", action="store_true",
                   help="text encoder on the song's stream (default: on a side stream, overlapping the "
                        "lyric / timbre encoders; the DiT starts only after all three)")
    p.add_argument("--repaint", action="store_true",
                   help="SURVEY config 5: VAE encode of a synthetic 48 kHz stereo source -> DiT repaint of "
                        "[--repaint-start, --repaint-end) s -> VAE decode, all inside the timed song")
    p.add_argument("--repaint-start", type=float, default=60.0)
    p.add_argument("--repaint-end", type=float, default=120.0)
    p.add_argument("--text-len", type=int, default=128)
    p.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc_roofline.json"),
                   help="counter passes of the roofline kernel (tools/pmc_roofline.py), spliced in LABELLED")
    p.add_argument("--dry-run", action="store_true",
                   help="CPU ranks over gloo with a stand-in song: exercises the launcher / timing / "
                        "max-over-ranks / JSON path without a GPU")
    p.add_argument("--no-output-leg", action="store_true",
                   help="skip the post-decode output leg measurement (D->H, PCM16 conversion, WAV write)")
    p.add_argument("--no-config1", action="store_true",
                   help="skip the CPU run of BASELINE config 1 (10 s turbo, 8 steps, fp32, in full)")
    return p.parse_args()


def host_cpus():
    """(threads to use, host CPU count, CPU model).  Threads = the CPUs this process
    may actually run on: its affinity set, capped by the cgroup CPU quota
    (cpu.max).  On the GPU box os.cpu_count() reports the whole host (256) while
    the job's quota is 16 CPUs; 256 threads on a 16-CPU quota would oversubscribe
    it and time the scheduler, not the math."""
    n_host = os.cpu_count() or 1
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = n_host
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            quota, period = open(path).read().split()[:2]
            if quota != "max":
                n = min(n, max(1, int(int(quota) // int(period))))
        except (OSError, ValueError):
            pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, n_host, model


def output_leg(pipe, song, dev, sec_per_song, n_songs=2):
    """SURVEY §8f row 4, measured after the timed region on rank 0: what happens to each song after
    the decode.  (a) the reference's host leg (inference.py:673-716, audio_utils.py:24-210): fp32
    D→H, normalize_audio on the host, the [samples, channels] PCM16 conversion soundfile applies,
    the file write; (b) acehip's leg run serially: guard + normalize + PCM16 pack fused on the GPU,
    D→H of the frames into pinned memory, the write; (c) (b) overlapped with the next songs (the
    AudioWriter: copy on a side stream, write on a host thread): songs/s with the leg against the
    timed line.  Files are PCM16 WAV via the stdlib `wave` module (soundfile / the FLAC encoder are
    not installed, so FLAC encoding itself is not timed)."""
    import tempfile
    from acehip.output import AudioWriter, postprocess_pcm16_, reference_host_leg, remove_quietly, write_wav_pcm16
    wav = pipe.wav
    B, C, N = wav.shape
    d = tempfile.mkdtemp(prefix="acehip_out_")
    paths = []
    try:
        ref = None
        for i in range(2):                      # the second run: warm page cache, like a serving loop
            p = os.path.join(d, f"ref{i}.wav")
            paths.append(p)
            r = reference_host_leg(wav[0], p)
            r.pop("frames")
            ref = r if ref is None or r["total_ms"] < ref["total_ms"] else ref
        host = torch.empty(N * C, dtype=torch.int16, pin_memory=True)
        best = None
        for i in range(2):
            w = wav[:1].clone()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            pcm = postprocess_pcm16_(w, -1.0)
            e1.record()
            host.copy_(pcm.view(-1), non_blocking=True)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            p = os.path.join(d, f"hip{i}.wav")
            paths.append(p)
            write_wav_pcm16(p, host.view(N, C), 48000, C)
            t2 = time.perf_counter()
            cur = {"gpu_pack_ms": e0.elapsed_time(e1), "pack_plus_d2h_ms": 1e3 * (t1 - t0), "write_ms": 1e3 * (t2 - t1),
                   "total_ms": 1e3 * (t2 - t0)}
            best = cur if best is None or cur["total_ms"] < best["total_ms"] else best
        writer = AudioWriter(dev, N, channels=C, slots=2)
        db, pipe.normalization_db = pipe.normalization_db, None    # the writer's fused pass normalizes
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        try:
            for i in range(n_songs):
                song(500 + i)
                p = os.path.join(d, f"song{i}.wav")
                paths.append(p)
                writer.submit(pipe.wav, [p])
            writer.flush()
            torch.cuda.synchronize()
            with_leg = (time.perf_counter() - t0) / n_songs
        finally:
            pipe.normalization_db = db
            writer.close()
    finally:
        remove_quietly(paths)
        try:
            os.rmdir(d)
        except OSError:
            pass
    return {
        "samples_per_song": N * C,
        "reference_host_leg_ms": {k: round(v, 2) for k, v in ref.items()},
        "reference_host_bytes_d2h": N * C * 4,
        "acehip_serial_leg_ms": {k: round(v, 3) for k, v in best.items()},
        "acehip_bytes_d2h": N * C * 2,
        "overlapped_s_per_song_with_leg": round(with_leg, 4),
        "overlapped_exposed_ms_per_song": round((with_leg - sec_per_song) * 1e3, 1),
        "note": "reference leg = fp32 D->H + host normalize_audio + [samples, channels] PCM16 conversion + "
                "WAV write (host torch on this job's CPU quota); acehip leg = fused GPU guard/normalize/PCM16 "
                "pack + pinned D->H of half the bytes + WAV write; overlapped = songs run back to back with the "
                "leg of song k (side-stream copy, writer thread) under song k+1 — exposed = its s/song minus "
                "the timed line's; FLAC encoding not timed (soundfile absent)",
    }


def cpu_baseline(W_gpu, cfg, vae_w, vcfg, T, lenc, Bc=2, n_steps=1):
    """Time the CPU oracle (PyTorch fp32) on a bounded sample and extrapolate."""
    from oracle import dit_oracle, vae_oracle
    threads, _, _ = host_cpus()
    torch.set_num_threads(threads)
    W = {k: v.detach().float().cpu() for k, v in W_gpu.items()}
    g = torch.Generator().manual_seed(0)
    S = (T + 1) // 2
    xt = torch.randn(Bc, T, 64, generator=g)
    ctx = torch.randn(Bc, T, 128, generator=g)
    enc = torch.randn(Bc, lenc, cfg.hidden_size, generator=g)
    t = torch.full((Bc,), 0.75)
    with torch.no_grad():
        kv = dit_oracle.cross_kv(W, cfg, enc)
        t0 = time.time()
        for _ in range(n_steps):   # n_steps > 1 only for the short song run in full
            dit_oracle.dit_forward(W, cfg, xt, t, t, enc, ctx, kv_cache=kv)
        dit_s = (time.time() - t0) / n_steps
    del W
    vae_s = 0.0
    win = T if n_steps > 1 else 64
    if vae_w is not None:
        Wv = {k: v.detach().float().cpu() for k, v in vae_w.items()}
        z = torch.randn(1, 64, win, generator=g)
        with torch.no_grad():
            t0 = time.time()
            vae_oracle.decode(Wv, vcfg, z)
            vae_s = time.time() - t0
    return {"dit_step_s": dit_s, "vae_window_s": vae_s, "threads": threads, "window": win}


def cpu_config1(W_gpu, cfg, lenc):
    """BASELINE config 1 run IN FULL on the host: DiT-only text2music, 10 s of audio
    (T = 250), the turbo 8-step table (shift 3), fp32, the PyTorch-CPU oracle
    (oracle/dit_oracle.py + oracle/sampler_oracle.py) on the bench's weights."""
    from oracle import dit_oracle, sampler_oracle
    threads, n_host, model = host_cpus()
    torch.set_num_threads(threads)
    W = {k: v.detach().float().cpu() for k, v in W_gpu.items()}
    g = torch.Generator().manual_seed(1)
    T = 250
    enc = torch.randn(1, lenc, cfg.hidden_size, generator=g)
    ctx = torch.cat([torch.randn(1, T, 64, generator=g), torch.ones(1, T, 64)], -1)
    noise = torch.randn(1, T, 64, generator=g)
    with torch.no_grad():
        t0 = time.time()
        kv = dit_oracle.cross_kv(W, cfg, enc)
        x = sampler_oracle.generate_turbo(lambda xt, tv: dit_oracle.dit_forward(W, cfg, xt, tv, tv, enc, ctx,
                                                                                kv_cache=kv), noise, shift=3.0)
        sec = time.time() - t0
    assert torch.isfinite(x).all()
    return {"value": round(sec, 2), "unit": "s/song", "cores": threads, "kind": "port", "cpu_model": model,
            "host_cpus": n_host,
            "config": "BASELINE configs[0]: DiT-only text2music, 10 s audio (T=250), turbo 8 steps shift 3, fp32 CPU",
            "sample": "the whole song in full (cross K/V once + 8 DiT forwards + turbo Euler/x0), not extrapolated"}


QWEN3_VOCAB = 151669   # Qwen3-Embedding-0.6B vocabulary


def dry_run(args, rank, world):
    """The multi-rank harness on CPU (gloo): same launch, barrier, timing, max-over-
    ranks and JSON as the GPU run, with a fixed stand-in song (a small fp32 matmul
    chain) — for the CPU test that --gpus N really yields N ranks."""
    from acehip import distributed as D
    torch.set_num_threads(1)
    D.init(backend="gloo")
    g = torch.Generator().manual_seed(1234)
    cond = torch.randn(64, 64, generator=g) if rank == 0 else torch.zeros(64, 64)
    t0 = time.time()
    D.broadcast_condition([cond])
    bcast_ms = (time.time() - t0) * 1e3
    ref = torch.randn(64, 64, generator=torch.Generator().manual_seed(1234))
    assert torch.equal(cond, ref), "conditioning broadcast mismatch"

    def song(seed):
        x = torch.randn(128, 128, generator=torch.Generator().manual_seed(seed))
        for _ in range(20):
            x = torch.tanh(x @ x.t() / 128)
        return x

    for i in range(args.warmup):
        song(10_000 + rank * 100 + i)
    D.barrier()
    t0 = time.time()
    for i in range(args.steps):
        song(rank * 1000 + i)
    D.barrier()
    elapsed_max = D.max_over_ranks(time.time() - t0)
    bc_all = D.gather_floats([bcast_ms])
    songs = args.steps * world
    if rank == 0:
        print(json.dumps({"metric": "seconds/song (dry run: CPU stand-in song)", "value": round(elapsed_max / songs, 6),
                          "unit": "s/song", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed_max / args.steps * 1e3, 3), "higher_is_better": False,
                          "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic (CPU dry run)",
                          "dry_run": True, "config": {"workload": "dry run", "global_batch": songs,
                                                      "parallelism": f"song-parallel x{world}"},
                          "ranks": world, "broadcast_ms_per_rank": [round(v, 3) for v in bc_all]}), flush=True)
    D.destroy()


def main():
    args = parse()
    from acehip import distributed as D
    if D.needs_launch(args.gpus):
        # one process per GPU: spawn the ranks before anything touches the GPU
        sys.exit(D.launch_local([os.path.abspath(__file__), *sys.argv[1:]], args.gpus))
    rank, world, local = D.env_world()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if args.dry_run:
        return dry_run(args, rank, world)
    from acehip.config import DiTConfig, VAEConfig
    from acehip.dit import AceStepDiTBackend, DiTRuntime
    from acehip.vae import OobleckBackend
    from acehip.weights import (synth_condenc_weights, synth_dit_weights, synth_null_condition,
                                synth_text_encoder_weights, synth_vae_weights)
    from acehip.condition import ConditionEncoder, HipPrepareCondition, TextEncoder
    from acehip.flops import dit_flops_executed_cfg_song_step, dit_flops_per_row, vae_decoder_flops
    from acehip.provenance import product_hash

    gi = local
    if os.environ.get("ACEHIP_DIST_BACKEND") == "gloo":
        # rehearsal of the multi-rank path on fewer GPUs than ranks (gloo, host-staged collectives)
        gi = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gi)
    dev = torch.device("cuda", gi)
    D.init(device=dev)

    T = int(round(args.seconds * 25))
    S = (T + 1) // 2
    cfg = DiTConfig()
    vcfg = VAEConfig()
    if args.turbo:
        args.guidance = 1.0
    do_cfg = args.guidance > 1.0
    Bc = 2 if do_cfg else 1

    # random-init weights of the real architecture, identical on every rank
    W = synth_dit_weights(cfg, seed=0, mode="bench", device=dev, dtype=torch.bfloat16, backend="torch")
    null = synth_null_condition(cfg, seed=0, device=dev, dtype=torch.bfloat16, backend="torch")
    rt = DiTRuntime(cfg, gi, max_S=S, max_Bc=Bc, max_Lenc=args.lenc)
    rt.load(W)
    rt.use_graph(args.graph)
    prep = None
    if not args.no_condition:
        # lyric + timbre + text encoders on the HIP path; Lenc = lyric + 1 timbre + text
        ce = ConditionEncoder(cfg, gi, max_batch=world, max_lyric=args.lyric_len, max_refs=world,
                              max_ref_frames=750)
        ce.load(synth_condenc_weights(cfg, seed=0, mode="bench", device=dev, dtype=torch.bfloat16, backend="torch"))
        prep = HipPrepareCondition(ce)
        args.lenc = args.lyric_len + 1 + args.text_len
        # the Qwen3-Embedding-0.6B text encoder (infer_text_embeddings / infer_lyric_embeddings,
        # conditioning_embed.py:71-79): 28 causal layers for the text tokens, the table for lyrics
        te_cfg = DiTConfig(**TextEncoder.QWEN3_06B)
        te = TextEncoder(te_cfg, gi, max_batch=world, max_tokens=max(args.text_len, 64),
                         overlap=not args.no_overlap)
        te.load(synth_text_encoder_weights(te_cfg, QWEN3_VOCAB, seed=0, mode="bench", device=dev,
                                           dtype=torch.bfloat16, backend="torch"))
    be = AceStepDiTBackend(rt, null, is_turbo=args.turbo, prepare_condition=prep)
    vae = vae_w = None
    if not args.no_vae:
        vae_w = synth_vae_weights(vcfg, seed=0, mode="bench", with_encoder=args.repaint, device=dev,
                                  dtype=torch.bfloat16, backend="torch")
        vae = OobleckBackend(vcfg, gi, max_T=T, with_encoder=args.repaint)
        vae.load(vae_w)

    # synthetic conditioning on rank 0, broadcast over RCCL; the
    # broadcasts are timed per rank (outside the timed song loop, like the reference's
    # batch preparation)
    bcast_ms = [0.0]

    def broadcast(ts):
        torch.cuda.synchronize()
        t0 = time.time()
        D.broadcast_condition(ts)
        torch.cuda.synchronize()
        bcast_ms[0] += (time.time() - t0) * 1e3
    g = torch.Generator(device=dev).manual_seed(1234)
    src = torch.randn(1, T, 64, device=dev, generator=g).bfloat16()          # silence latents
    chunk = torch.ones(1, T, 64, device=dev).bfloat16()
    if args.no_condition:
        enc = torch.randn(1, args.lenc, cfg.hidden_size, device=dev, generator=g).bfloat16()
        ctx = torch.cat([src, chunk], dim=-1).contiguous()
        broadcast([enc, ctx])
        cond_kw = dict(encoder_hidden_states=enc, context_latents=ctx)
    else:
        # text / lyric token ids and a 30 s timbre reference; the text encoder and the
        # condition encoders (prepare_condition, base:1607-1652) run inside the timed song
        text_ids = torch.randint(0, QWEN3_VOCAB, (1, args.text_len), device=dev, generator=g)
        lyric_ids = torch.randint(0, QWEN3_VOCAB, (1, args.lyric_len), device=dev, generator=g)
        refer = torch.randn(1, 750, cfg.timbre_hidden_dim, device=dev, generator=g).bfloat16()
        broadcast([text_ids, lyric_ids, refer, src])
        cond_kw = dict(text_attention_mask=torch.ones(1, args.text_len, device=dev, dtype=torch.long),
                       lyric_attention_mask=torch.ones(1, args.lyric_len, device=dev, dtype=torch.long),
                       refer_audio_acoustic_hidden_states_packed=refer,
                       refer_audio_order_mask=torch.zeros(1, device=dev, dtype=torch.long),
                       src_latents=src, chunk_masks=chunk, is_covers=torch.zeros(1, device=dev, dtype=torch.long))

    span = None
    if args.repaint:
        assert vae is not None and not args.no_condition, "--repaint needs the VAE and the condition encoders"
        # synthetic source: 3 seeded sines + N(0, 0.05), peak −12 dBFS
        n = T * vcfg.hop_length
        tt = torch.arange(n, device=dev, dtype=torch.float32) / 48000.0
        sw = sum(torch.sin(2 * math.pi * f * tt + ph) for f, ph in ((220.0, 0.1), (330.0, 0.7), (523.25, 1.9)))
        sw = torch.stack([sw, torch.roll(sw, 480)])[None]
        sw = sw + 0.05 * torch.randn(sw.shape, device=dev, generator=g)
        src_wav = (sw / sw.abs().amax() * 10 ** (-12 / 20)).bfloat16().contiguous()
        del sw, tt
        broadcast([src_wav])
        # conditioning_masks.py:37-50: latent span [start·48000//1920, end·48000//1920)
        span = (int(args.repaint_start * 48000 // 1920), int(args.repaint_end * 48000 // 1920))
        span_mask = torch.zeros(1, T, 64, device=dev, dtype=torch.bfloat16)
        span_mask[:, span[0]:span[1]] = 1

    if span is not None and world > 1:
        raise SystemExit("bench.py: --repaint is the 1-GPU config 5 (SURVEY §8d); run it with --gpus 1")
    # song-parallel: rank 0 conditions the step's batch of `world` songs once
    # (text encoder + prepare_condition in one batched pass) and draws the batch noise, each rank
    # gets its song by scatter, runs generate_audio + the VAE decode on its own GPU, and the
    # latents return to rank 0; at world 1 the scatter / gather are the identity
    pipe = D.SongParallelPipeline(be, vae, device=dev, gather_wav=False)
    pipe.timing = True

    def batch_kwargs(seeds):
        Bw = len(seeds)
        if args.no_condition:
            return dict(encoder_hidden_states=enc.expand(Bw, -1, -1).contiguous(),
                        context_latents=ctx.expand(Bw, -1, -1).contiguous(), seed=seeds)
        kw = {k: v.expand(Bw, *v.shape[1:]).contiguous() for k, v in cond_kw.items()}
        kw["refer_audio_order_mask"] = torch.arange(Bw, device=dev, dtype=torch.long)
        kw.update(text_hidden_states=te(input_ids=text_ids.expand(Bw, -1).contiguous(),
                                        lyric_attention_mask=None).last_hidden_state,
                  lyric_hidden_states=te.embed_tokens(lyric_ids.expand(Bw, -1).contiguous()), seed=seeds)
        return kw

    def song(idx, warm=False):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        seeds = [(10_000 + r * 100 + idx) if warm else (r * 1000 + idx) for r in range(world)]
        if span is not None:
            # vae.encode(x).latent_dist.sample() (vae_encode.py:65), then the repaint source:
            # encoded target with silence inside the span + chunk mask of the span
            # (conditioning_masks.py:67-83), through the handler seam as the reference calls it
            # (batch_prep.py:63-76: tiled_encode(audio, offload_latent_to_cpu=True) → .to(device))
            z = vae.tiled_encode(src_wav, offload_latent_to_cpu=True).to(dev).transpose(1, 2)
            src_r = z.clone()
            src_r[:, span[0]:span[1]] = src[:, span[0]:span[1]]
            cond_kw.update(src_latents=src_r.contiguous(), chunk_masks=span_mask)
        sampler = dict(infer_steps=args.infer_steps, diffusion_guidance_sale=args.guidance, shift=args.shift,
                       infer_method="ode")
        if rank == 0:
            pipe.generate(**batch_kwargs(seeds), **sampler)
        else:
            pipe.serve_one()
        e1, e2 = pipe.last_events
        return e0, e1, e2

    for i in range(args.warmup):
        song(i, warm=True)
    torch.cuda.synchronize()
    # inside the timed region only the roofline kernel carries events
    rt.profile(True, kinds=["gemm_swiglu"])
    D.barrier(dev)
    torch.cuda.synchronize()
    t0 = time.time()
    evs = [song(i) for i in range(args.steps)]
    torch.cuda.synchronize()
    D.barrier(dev)
    elapsed = time.time() - t0
    elapsed_max = D.max_over_ranks(elapsed, dev)
    prof = rt.profile_read()
    # per-kernel breakdown from one extra, untimed song with every family timed
    rt.profile(True)
    song(999)
    torch.cuda.synchronize()
    prof_all = rt.profile_read()
    rt.profile(False)
    dit_ms = sum(a.elapsed_time(b) for a, b, _ in evs) / args.steps
    vae_ms = sum(b.elapsed_time(c) for _, b, c in evs) / args.steps

    songs = args.steps * world
    sec_per_song = elapsed_max / songs
    bcast_all = D.gather_floats([bcast_ms[0]], dev)
    dit_flops_song = args.infer_steps * Bc * dit_flops_per_row(cfg, S, args.lenc)
    # what the HIP path executes: the CFG null rows' cross-attention block and the
    # layer-0 dedup are skipped algebraically (acehip.flops)
    dit_flops_exec = (args.infer_steps * dit_flops_executed_cfg_song_step(cfg, S, args.lenc) if Bc == 2
                      else dit_flops_song)
    vae_flops_song = vae_decoder_flops(vcfg, T) if vae is not None else 0.0
    M = Bc * S
    n_sw, ms_sw = prof["gemm_swiglu"]
    sw_flops = 2.0 * M * (2 * cfg.intermediate_size) * cfg.hidden_size
    sw_ms = ms_sw / max(n_sw, 1)
    sw_tflops = sw_flops / (sw_ms * 1e-3) / 1e12 if n_sw else None
    # algorithmic bytes of one SwiGLU call: A [M][K] + W [N][K] in, C [M][N/2] out (bf16)
    sw_N, sw_K = 2 * cfg.intermediate_size, cfg.hidden_size
    sw_bytes = 2.0 * (M * sw_K + sw_N * sw_K + M * sw_N // 2)
    kname = "SwiGLU gate/up GEMM, EPI_SWIGLU (M=%d N=%d K=%d)" % (M, sw_N, sw_K)
    if sw_flops / sw_bytes >= PEAK_BF16_TFLOPS / PEAK_HBM_GBS * 1e3:     # above the ridge: MFMA-bound
        roofline = {"bound": "mfma", "kernel": kname, "achieved": round(sw_tflops, 1) if sw_tflops else None,
                    "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(sw_tflops / PEAK_BF16_TFLOPS, 4) if sw_tflops else None}
    else:   # short songs: the weight stream dominates (arithmetic intensity below the ridge)
        gbs = sw_bytes / (sw_ms * 1e-3) / 1e9 if n_sw else None
        roofline = {"bound": "hbm", "kernel": kname, "achieved": round(gbs, 1) if gbs else None,
                    "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4) if gbs else None,
                    "algorithmic_bytes": sw_bytes}
    roofline.update({"avg_launch_us": round(sw_ms * 1e3, 1), "launches": n_sw, "traffic": None})
    # HBM traffic (FETCH_SIZE / WRITE_SIZE) and MFMA-busy / clock (SQ / GRBM) of this kernel
    # come from SEPARATE rocprofv3 --pmc passes (counters cannot be read inside this timed
    # run); they are spliced in only for the same GEMM shape and labelled with the file
    # they come from and the box / clock / tree they were measured on — never as this run's
    # numbers (tools/pmc_roofline.py writes the file from the passes)
    try:
        with open(args.pmc_json) as f:
            pm = json.load(f)
        sw = pm.get("gemm_swiglu") or {}
        if sw.get("M") == M:
            roofline["traffic"] = sw.get("hbm_bytes_per_call")
            roofline["pmc_from"] = {
                "file": os.path.relpath(args.pmc_json, REPO), "same_run": False,
                "box": pm.get("box"), "git_head": pm.get("git_head"),
                "product_hash": pm.get("product_hash"),
                "same_product_code": pm.get("product_hash") == product_hash(),
                "clock_GHz": sw.get("clock_GHz"), "mfma_busy_frac": sw.get("mfma_busy_frac"),
                "avg_us_in_pass": sw.get("avg_us"),
                "note": "counter passes of the same kernel shape on the named box (separate runs); "
                        "traffic = FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE per call"}
    except Exception:
        pass
    kernels = {k: {"launches": n, "avg_us": (ms / n * 1e3 if n else None)} for k, (n, ms) in prof_all.items()}

    out = {
        "metric": f"seconds/song ({args.seconds:g} s audio, {args.infer_steps} DiT steps)",
        "value": round(sec_per_song, 4),
        "unit": "s/song",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max / args.steps * 1e3, 2),
        "higher_is_better": False,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (random-init weights of the real architecture, random conditioning)",
        "config": {"workload": f"text2music {args.seconds:g}s, "
                               + (f"turbo {args.infer_steps} steps (table, no CFG), " if args.turbo else
                                  f"base/sft {args.infer_steps} steps, shift {args.shift:g}, CFG {args.guidance:g} + APG, ")
                               + ("DiT + VAE decode" if args.no_condition else "text encoder + condition encoders + DiT + VAE decode")
                               + (f", repaint [{args.repaint_start:g}, {args.repaint_end:g}) s: VAE encode first"
                                  if args.repaint else ""),
                   "global_batch": songs, "seq_len": S, "latent_frames": T, "lenc": args.lenc,
                   "parallelism": f"song-parallel x{world}"},
        "songs_per_s": round(songs / elapsed_max, 4),
        "dit_ms_per_song": round(dit_ms, 2),
        "dit_ms_note": "generate_audio wall on the GPU stream: (repaint: VAE encode +) condition encoders (once) + CFG DiT steps",
        "dit_ms_per_step": round(dit_ms / args.infer_steps, 3),
        "vae_ms_per_song": round(vae_ms, 2),
        "dit_tflops_effective": round(dit_flops_song / (dit_ms * 1e-3) / 1e12, 1),
        "dit_mfma_frac_effective": round(dit_flops_song / (dit_ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
        "dit_tflops_executed": round(dit_flops_exec / (dit_ms * 1e-3) / 1e12, 1),
        "dit_mfma_frac_executed": round(dit_flops_exec / (dit_ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
        "dit_flops_note": "effective = the reference's algorithmic DiT FLOPs (SURVEY §8d) / DiT time; executed = "
                          "the FLOPs the HIP path runs (CFG null-row cross-attention block and layer-0 CFG dedup "
                          "skipped algebraically, -8.5 % at 240 s) / DiT time; both include the condition encoders' "
                          "time in the denominator",
        "broadcast_ms_per_rank": [round(v, 3) for v in bcast_all],
        "vae_tflops": round(vae_flops_song / (vae_ms * 1e-3) / 1e12, 1) if vae is not None else None,
        "roofline": roofline,
        "kernels": kernels,
        "kernels_note": "per-launch averages (HIP events on the forward stream) from one extra untimed song; the timed region carries events only around the roofline kernel",
    }
    if rank == 0 and world == 1 and vae is not None and not args.no_output_leg:
        leg = output_leg(pipe, song, dev, sec_per_song)
        out["output_ms_per_song"] = leg["acehip_serial_leg_ms"]["total_ms"]
        out["output_leg"] = leg
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # a short song (10 s, 8 turbo steps) runs in full; longer ones
        # time one DiT step + one 64-frame VAE window and extrapolate
        full = T <= 250
        cb = cpu_baseline(W, cfg, vae_w, vcfg, T, args.lenc, Bc=Bc, n_steps=args.infer_steps if full else 1)
        n_win = math.ceil(T / cb["window"])
        sec = cb["dit_step_s"] * args.infer_steps + cb["vae_window_s"] * n_win
        kind = "CFG " if Bc == 2 else ""
        sample = (f"the whole song: {args.infer_steps} {kind}DiT steps (Bc={Bc}, S={S}, {cb['dit_step_s']:.2f}s each) "
                  f"+ the {T}-frame VAE decode ({cb['vae_window_s']:.2f}s); fp32 PyTorch-CPU oracle, not extrapolated"
                  if full else
                  f"1 full-size {kind}DiT step (Bc={Bc}, S={S}) = {cb['dit_step_s']:.2f}s x {args.infer_steps} "
                  f"+ one {cb['window']}-frame VAE decode window = {cb['vae_window_s']:.2f}s x {n_win}; "
                  f"fp32 PyTorch-CPU oracle, extrapolated")
        n_thr, n_host, model = host_cpus()
        out["cpu_baseline"] = {"value": round(sec, 2 if full else 1), "unit": "s/song", "cores": cb["threads"],
                               "kind": "port", "sample": sample, "cpu_model": model, "host_cpus": n_host,
                               "cores_note": f"threads = this job's CPU quota ({n_thr} of the host's {n_host} "
                                             "CPUs; the cgroup cpu.max caps it, more threads would only "
                                             "oversubscribe the quota)"}
        if not args.no_config1:
            out["cpu_baseline_config1"] = cpu_config1(W, cfg, args.lenc)
    if rank == 0:
        print(json.dumps(out), flush=True)
    D.destroy()


if __name__ == "__main__":
    main()
