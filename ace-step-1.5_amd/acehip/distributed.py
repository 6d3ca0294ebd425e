"""Song-parallel multi-GPU plumbing.

The denoise loop and the VAE decode of one song never talk to another song
(per-seed noise base:1749-1763, APG norms per (song, channel) apg_guidance.py
:27-28,49), so the node is partitioned song-per-GPU, one process per GPU, with
``torch.distributed`` backend ``"nccl"`` (= RCCL over xGMI on ROCm).  The
only collectives are outside the denoise step:
  * a broadcast of the per-batch conditioning from rank 0 (enc [1,Lenc,2048]
    bf16 ≈ 2.6 MB, context [1,T,128] ≈ 1.5 MB at 240 s — tens of µs per link);
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
            backend = "nccl" if torch.cuda.is_available() else "gloo"
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
        dist.broadcast(t, src=src)


def max_over_ranks(x: float, device: Optional[torch.device] = None) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device: Optional[torch.device] = None):
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if device is not None and device.type == "cuda":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def gather_floats(vals: Sequence[float], device: Optional[torch.device] = None) -> List[float]:
    """All ranks' values, rank-major (all_gather; the caller's own list at world 1)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(v) for v in vals]
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x) for o in out for x in o.tolist()]


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def gather_to_rank0(t: torch.Tensor) -> Optional[List[torch.Tensor]]:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [t]
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())] if dist.get_rank() == 0 else None
    dist.gather(t, out, dst=0)
    return out
