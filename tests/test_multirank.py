"""Multi-rank CPU tests of the song-parallel path through the SAME
launcher bench.py uses (acehip.distributed.launch_local): gloo ranks on this
host, conditioning broadcast, rank-sharded songs, max-over-ranks; and bench.py
itself: ``--gpus N`` really runs N ranks (spawned, or under torchrun), and a
launcher/--gpus mismatch is refused."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

from acehip import distributed as D

WORKER = os.path.join(REPO, "tests", "helpers", "dist_worker.py")


def _last_json(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


@pytest.mark.parametrize("world", [2, 3])
def test_launch_local_song_parallel(tmp_path, world):
    rc = D.launch_local([WORKER], world, extra_env={"ACEHIP_TEST_OUT": str(tmp_path)}, timeout=180)
    assert rc == 0
    recs = sorted((json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)), key=lambda r: r["rank"])
    assert [r["rank"] for r in recs] == list(range(world))
    for r in recs:
        assert r["world"] == world and r["local"] == r["rank"]
        assert r["enc_sum"] == sum(range(40)) and r["ctx_sum"] == 84.0      # rank 0's condition everywhere
        assert r["max"] == 10.0 * (world - 1)
    assert sorted(s for r in recs for s in r["songs"]) == list(range(6))    # every song on exactly one rank
    assert recs[0]["all_songs_once"]


def test_launch_local_propagates_failure():
    code = "import os, sys, time; r = int(os.environ['RANK']); time.sleep(0.2 * r); sys.exit(3 if r == 1 else 0)"
    assert D.launch_local(["-c", code], 2, timeout=60) == 3


def test_needs_launch(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert D.needs_launch(2) and not D.needs_launch(1)
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert not D.needs_launch(2)


def _bench(args, env=None, timeout=240):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.pop("RANK", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          env=e, timeout=timeout)


def test_bench_gpus2_spawns_two_ranks():
    p = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    j = _last_json(p.stdout)
    assert j["n_gpus"] == 2 and j["ranks"] == 2 and j["config"]["global_batch"] == 4
    assert len(j["broadcast_ms_per_rank"]) == 2


def test_bench_under_torchrun():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(29600 + os.getpid() % 300),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "0", "--dry-run"]
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    p = subprocess.run(cmd, capture_output=True, text=True, env=e, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    j = _last_json(p.stdout)
    assert j["n_gpus"] == 2 and j["config"]["global_batch"] == 4


def test_bench_refuses_world_mismatch():
    p = _bench(["--gpus", "4", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=2" in (p.stderr + p.stdout)


PIPE_WORKER = os.path.join(REPO, "tests", "helpers", "pipeline_worker.py")


@pytest.mark.parametrize("world", [2, 3])
def test_song_parallel_pipeline(tmp_path, world):
    """SongParallelPipeline: rank 0 conditions the batch once, draws the batch
    noise, scatters per song; every rank runs its songs; latents gathered in batch order —
    equal to the single-process batch for an int seed (one generator), per-song seeds with
    cover noise, and acs < 1 with fewer songs than ranks; the serve loop ends on stop()."""
    rc = D.launch_local([PIPE_WORKER], world, extra_env={"ACEHIP_TEST_OUT": str(tmp_path)}, timeout=180)
    assert rc == 0
    recs = {r: json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)}
    assert recs[0]["ok"] == [True, True, True, True, True]
    # song i on rank i % world: batch sizes 5, 4, 1 (then 1, 5 with the VAE) split round-robin;
    # idle ranks run nothing
    for r in range(world):
        want = [n for n in (len(D.song_assignment(B, r, world)) for B in (5, 4, 1, 1, 5)) if n]
        assert recs[r]["calls"] == want, (r, recs[r]["calls"], want)
