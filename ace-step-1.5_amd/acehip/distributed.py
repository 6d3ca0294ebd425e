"""Song-parallel multi-GPU plumbing.

The denoise loop and the VAE decode of one song never talk to another song
(per-seed noise base:1749-1763, APG norms per (song, channel) apg_guidance.py
:27-28,49), so the node is partitioned song-per-GPU, one process per GPU, with
``torch.distributed`` backend ``"nccl"`` (= RCCL over xGMI on ROCm).  The
only collectives are outside the denoise step:
  * rank 0 conditions the whole batch once and scatters each song's encoder states
    (enc [1,Lenc,2048] bf16 ≈ 2.6 MB), context [1,T,128] ≈ 1.5 MB and noise [1,T,64]
    ≈ 0.77 MB at 240 s — tens of µs per link (:class:`SongParallelPipeline`);
  * a MAX all-reduce of the timed region for the bench;
  * optional gather of results (latents 0.77 MB / song) to rank 0.
Scaling is therefore "weak": per-GPU work is fixed as the node grows.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), \
        int(os.environ.get("LOCAL_RANK", 0))


def needs_launch(n_procs: int) -> bool:
    """True when ``n_procs`` > 1 ranks are asked for but this process was not
    started by a launcher (no WORLD_SIZE in the environment)."""
    return n_procs > 1 and "WORLD_SIZE" not in os.environ


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_local(argv: Sequence[str], n_procs: int, extra_env: Optional[dict] = None,
                 timeout: Optional[float] = None) -> int:
    """Start ``n_procs`` ranks of ``python argv...`` on this node — one process per
    GPU, the torchrun environment contract (RANK / LOCAL_RANK / WORLD_SIZE /
    LOCAL_WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT) — and wait for all.

    Must be called before anything touches the GPU (the children are fresh
    interpreters started with subprocess, never exec).  If a rank fails, the
    remaining ranks are terminated (by their exact PIDs) and its exit code is
    returned; 0 when every rank succeeded."""
    port = _free_port()
    procs = []
    for r in range(n_procs):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n_procs),
                    "LOCAL_WORLD_SIZE": str(n_procs), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
        env.update(extra_env or {})
        procs.append(subprocess.Popen([sys.executable, *argv], env=env))
    deadline = None if timeout is None else time.time() + timeout
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:                 # one rank died: end the others
                    q.send_signal(signal.SIGTERM)
        if deadline is not None and time.time() > deadline and live:
            for q in live:
                q.kill()
            rc = rc or 124
            deadline = None
        time.sleep(0.05)
    return rc


def init(backend: Optional[str] = None, device: Optional[torch.device] = None):
    """Initialise the process group from torchrun's env (no-op at world 1)."""
    rank, world, local = env_world()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = os.environ.get("ACEHIP_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        kw = {}
        if backend == "nccl" and device is not None:
            kw["device_id"] = device
        dist.init_process_group(backend=backend, **kw)
    return rank, world, local


def song_assignment(n_songs: int, rank: int, world: int) -> List[int]:
    """Song i → rank i % world (round-robin; equal counts when world | n)."""
    return [i for i in range(n_songs) if i % world == rank]


def broadcast_condition(tensors: Sequence[torch.Tensor], src: int = 0) -> None:
    """In-place broadcast of the conditioning tensors from ``src``."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    for t in tensors:
        c = comm_device(t.device)
        if c is not None and c != t.device:
            h = t.to(c)
            dist.broadcast(h, src=src)
            t.copy_(h)
        else:
            dist.broadcast(t, src=src)


def comm_device(device: Optional[torch.device]) -> Optional[torch.device]:
    """Where collective buffers live: the GPU under RCCL, host memory under gloo (which moves
    CPU tensors only — the ``ACEHIP_DIST_BACKEND=gloo`` rehearsal of the multi-rank path with
    several ranks on one GPU)."""
    if dist.is_available() and dist.is_initialized() and dist.get_backend() == "gloo":
        return torch.device("cpu")
    return device


def max_over_ranks(x: float, device: Optional[torch.device] = None) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=comm_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device: Optional[torch.device] = None):
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if device is not None and device.type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def gather_floats(vals: Sequence[float], device: Optional[torch.device] = None) -> List[float]:
    """All ranks' values, rank-major (all_gather; the caller's own list at world 1)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(v) for v in vals]
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=comm_device(device))
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x) for o in out for x in o.tolist()]


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def _dist_world() -> tuple:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class SongParallel:
    """Batch plumbing for songs spread over the node, one process per GPU.

    ``scatter`` sends each rank the rows of per-song batch tensors that belong to its songs
    (song ``i`` → rank ``i % world``, ``song_assignment``) plus a small metadata object;
    ``gather`` returns per-song results to rank 0 in batch order.  Messages: one
    ``broadcast_object_list`` (batch size, shapes, dtypes, metadata), then one ``scatter`` per
    tensor of ``[k, ...]`` slots per rank with k = ⌈B / world⌉ (unused slots zero, never
    read).  At world 1 both calls are the identity."""

    def __init__(self, device: Optional[torch.device] = None):
        self.rank, self.world = _dist_world()
        self.device = device
        self._B = None

    def scatter(self, tensors: Optional[Sequence[Optional[torch.Tensor]]] = None, meta=None):
        """Rank 0 passes ``tensors`` (each [B, ...] or None) and ``meta`` (any picklable
        object); the other ranks pass nothing.  Every rank gets ``(songs, parts, meta)``: its
        batch indices, the rows of each tensor for those songs (None stays None), and meta."""
        if self.world == 1:
            ts = list(tensors)
            self._B = next(t.shape[0] for t in ts if t is not None)
            return list(range(self._B)), ts, meta
        dev, cdev = self.device, comm_device(self.device)
        if self.rank == 0:
            ts = list(tensors)
            B = next(t.shape[0] for t in ts if t is not None)
            assert all(t is None or t.shape[0] == B for t in ts), [None if t is None else t.shape for t in ts]
            hdr = [B, [None if t is None else (tuple(t.shape[1:]), t.dtype) for t in ts], meta]
        else:
            hdr = [None, None, None]
        dist.broadcast_object_list(hdr, src=0, device=cdev)
        B, specs, meta = hdr
        k = -(-B // self.world)
        mine = song_assignment(B, self.rank, self.world)
        parts = []
        for j, spec in enumerate(specs):
            if spec is None:
                parts.append(None)
                continue
            shape, dtype = spec
            recv = torch.empty(k, *shape, device=cdev, dtype=dtype)
            send = None
            if self.rank == 0:
                full = ts[j].to(cdev)
                send = []
                for r in range(self.world):
                    p = torch.zeros(k, *shape, device=cdev, dtype=dtype)
                    idx = song_assignment(B, r, self.world)
                    if idx:
                        p[:len(idx)] = full[idx]
                    send.append(p)
            dist.scatter(recv, send, src=0)
            parts.append(recv[:len(mine)].to(dev) if dev is not None else recv[:len(mine)])
        self._B = B
        return mine, parts, meta

    def gather(self, t: torch.Tensor) -> Optional[torch.Tensor]:
        """This rank's per-song results [c, ...] (its songs, in ``scatter`` order) → rank 0 gets
        the whole batch [B, ...] in batch order; the other ranks get None."""
        if self.world == 1:
            return t
        B = self._B
        k = -(-B // self.world)
        cdev = comm_device(t.device)
        buf = torch.zeros(k, *t.shape[1:], device=cdev, dtype=t.dtype)
        buf[:t.shape[0]] = t
        parts = [torch.empty_like(buf) for _ in range(self.world)] if self.rank == 0 else None
        dist.gather(buf, parts, dst=0)
        if self.rank != 0:
            return None
        out = torch.empty(B, *t.shape[1:], device=cdev, dtype=t.dtype)
        for r in range(self.world):
            idx = song_assignment(B, r, self.world)
            if idx:
                out[idx] = parts[r][:len(idx)]
        return out.to(t.device)


# sampler keyword arguments forwarded to every rank (the rest of the generate_audio contract,
# service_generate_execute.py:62-105, is conditioning, which rank 0 turns into tensors)
_SAMPLER_KW = ("infer_steps", "diffusion_guidance_sale", "shift", "infer_method", "use_adg", "cfg_interval_start",
               "cfg_interval_end", "audio_cover_strength", "cover_noise_strength", "timesteps")
# generate_audio keywords rank 0 consumes into the scattered tensors (conditioning, noise seed)
_CONDITION_KW = ("text_hidden_states", "text_attention_mask", "lyric_hidden_states", "lyric_attention_mask",
                 "refer_audio_acoustic_hidden_states_packed", "refer_audio_order_mask", "src_latents", "chunk_masks",
                 "is_covers", "silence_latent", "attention_mask", "seed", "non_cover_text_hidden_states",
                 "non_cover_text_attention_mask", "precomputed_lm_hints_25Hz", "audio_codes",
                 "encoder_hidden_states", "encoder_attention_mask", "context_latents")


def _rank_kwargs(kw: dict) -> dict:
    """The keywords every rank's generate_audio gets: the sampler keywords plus any other
    non-tensor keyword the caller passed (e.g. turbo's ``fix_nfe``, ``use_progress_bar``), so a
    call behaves the same through the pipeline as on ``AceStepDiTBackend.generate_audio``
    directly.  An unknown TENSOR keyword cannot be split per song and is refused."""
    meta = {}
    for k, v in kw.items():
        if k in _CONDITION_KW:
            continue
        if k == "timesteps" and isinstance(v, torch.Tensor):
            v = v.tolist()
        elif isinstance(v, torch.Tensor):
            raise TypeError(f"SongParallelPipeline: tensor keyword {k!r} is neither conditioning nor a sampler "
                            "argument; it cannot be split per song")
        meta[k] = v
    return meta


class SongParallelPipeline:
    """``generate_audio`` (+ the VAE decode) of one request's songs across the node.

    Rank 0 calls :meth:`generate` with the reference's ``generate_audio`` keyword arguments for
    the whole batch (``base:1783-1813``); every other rank calls :meth:`serve` (a loop) or
    :meth:`serve_one`.  Rank 0 runs the batch's conditioning once — ``prepare_condition`` over
    all B songs in one pass (the reference's ``base:1820``), the non-cover condition when
    ``audio_cover_strength < 1`` — and draws the batch noise with the reference's
    ``prepare_noise`` (so an int seed's single batch generator is honoured exactly), then
    scatters per song: encoder states, context latents, noise (and ``src_latents`` for cover
    noise).  Each rank runs its songs through ``AceStepDiTBackend.generate_audio`` and, with a
    VAE, decodes them (+ the output guard / normalisation) on its own GPU: no collective inside
    the denoise loop or the decode.  Latents (0.77 MB per 240 s song) return to rank 0;
    audio (92 MB per song) only when ``gather_wav``."""

    def __init__(self, dit, vae=None, device: Optional[torch.device] = None, gather_wav: bool = False,
                 normalization_db: Optional[float] = -1.0):
        self.dit, self.vae = dit, vae
        self.sp = SongParallel(device)
        self.gather_wav = gather_wav
        self.normalization_db = normalization_db
        self.wav = None              # this rank's decoded songs after the last call
        self.timing = False          # record (after generate_audio, after decode) CUDA events
        self.last_events = None

    def generate(self, **kw) -> dict:
        """Rank 0 only.  Returns ``{"target_latents": [B,T,64], "time_costs", "songs",
        "wav"}`` — ``wav`` is the whole batch when ``gather_wav``, else rank 0's own songs."""
        assert self.sp.rank == 0, "SongParallelPipeline.generate runs on rank 0 (the others serve())"
        be = self.dit
        enc, _mask, ctx = be._condition(kw)
        dtype, dev = be.dtype, be.device
        enc = enc.to(dev, dtype)
        ctx = ctx.to(dev, dtype).contiguous()
        B, T = ctx.shape[0], ctx.shape[1]
        from .dit import prepare_noise
        noise = prepare_noise((B, T, ctx.shape[-1] // 2), dev, dtype, kw.get("seed"))
        enc_nc = ctx_nc = None
        if float(kw.get("audio_cover_strength", 1.0)) < 1.0:
            enc_nc, _, ctx_nc = be._non_cover_condition(kw, ctx)
            enc_nc, ctx_nc = enc_nc.to(dev, dtype), ctx_nc.to(dev, dtype)
        src = kw.get("src_latents") if float(kw.get("cover_noise_strength", 0.0)) > 0.0 else None
        meta = _rank_kwargs(kw)
        return self._run([enc, ctx, noise, None if src is None else src.to(dev, dtype), enc_nc, ctx_nc], meta)

    def serve_one(self) -> None:
        """Ranks > 0: take part in one ``generate`` of rank 0."""
        assert self.sp.rank != 0
        self._run(None, None)

    def serve(self, n: Optional[int] = None) -> None:
        """Ranks > 0: serve ``n`` requests (forever when None; rank 0 ends it with :meth:`stop`)."""
        i = 0
        while n is None or i < n:
            if not self._run(None, None, allow_stop=True):
                return
            i += 1

    def stop(self) -> None:
        """Rank 0: release ranks looping in :meth:`serve`."""
        if self.sp.world > 1:
            dist.broadcast_object_list(["stop", None, None], src=0, device=comm_device(self.sp.device))

    def _run(self, tensors, meta, allow_stop=False):
        sp = self.sp
        if sp.world > 1 and sp.rank != 0:
            hdr = [None, None, None]
            dist.broadcast_object_list(hdr, src=0, device=comm_device(sp.device))     # "go" / "stop"
            if hdr[0] == "stop":
                assert allow_stop
                return False
        elif sp.world > 1:
            dist.broadcast_object_list(["go", None, None], src=0, device=comm_device(sp.device))
        songs, parts, meta = sp.scatter(tensors, meta)
        enc, ctx, noise, src, enc_nc, ctx_nc = parts
        kw = dict(meta)
        if isinstance(kw.get("timesteps"), list):
            kw["timesteps"] = torch.tensor(kw["timesteps"], dtype=torch.float32, device=self.dit.device)
        if src is not None:
            kw["src_latents"] = src
        if enc_nc is not None:
            kw["_non_cover"] = (enc_nc, ctx_nc)
        if songs:
            res = self.dit.generate_audio(encoder_hidden_states=enc, context_latents=ctx.contiguous(),
                                          _noise=noise, **kw)
            lat = res["target_latents"]
            costs = res["time_costs"]
        else:                         # more ranks than songs: nothing to do on this one
            lat = torch.zeros(0, ctx.shape[1], noise.shape[-1], device=noise.device, dtype=noise.dtype)
            costs = {}
        e_dit = e_vae = None
        if self.timing:
            e_dit = torch.cuda.Event(enable_timing=True)
            e_dit.record()
        wav = None
        if self.vae is not None and songs:
            wav = self.vae.decode_tensor(lat.transpose(1, 2))
            if self.normalization_db is not None:
                self.vae.postprocess_(wav, normalization_db=self.normalization_db)
        self.wav = wav
        if self.timing:
            e_vae = torch.cuda.Event(enable_timing=True)
            e_vae.record()
            self.last_events = (e_dit, e_vae)
        all_lat = sp.gather(lat)
        all_wav = wav
        if self.gather_wav and self.vae is not None:
            if wav is None:           # a rank without songs still joins the collective
                c = self.vae.cfg
                wav = torch.zeros(0, c.audio_channels, lat.shape[1] * c.hop_length, device=lat.device,
                                  dtype=torch.float32)
            all_wav = sp.gather(wav)
        if sp.rank == 0:
            return {"target_latents": all_lat, "time_costs": costs, "songs": songs, "wav": all_wav}
        return True


def gather_to_rank0(t: torch.Tensor) -> Optional[List[torch.Tensor]]:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [t]
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())] if dist.get_rank() == 0 else None
    dist.gather(t, out, dst=0)
    return out
