"""One rank of the multi-rank CPU test (started by acehip.distributed.launch_local):
gloo process group from the launcher's environment, conditioning broadcast from
rank 0, rank-sharded songs (song i -> rank i % world), max-over-ranks, gather to
rank 0.  Writes its observations as JSON to $ACEHIP_TEST_OUT/rank<r>.json."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ace-step-1.5_amd")]

import torch  # noqa: E402

from acehip import distributed as D  # noqa: E402

N_SONGS = 6


def main():
    torch.set_num_threads(1)
    rank, world, local = D.init(backend="gloo")
    enc = torch.full((1, 5, 8), float(rank))
    ctx = torch.full((1, 7, 4), float(rank) + 0.5)
    if rank == 0:
        enc = torch.arange(40, dtype=torch.float32).reshape(1, 5, 8)
        ctx = torch.ones(1, 7, 4) * 3
    D.broadcast_condition([enc, ctx])
    mine = D.song_assignment(N_SONGS, rank, world)
    # a stand-in "song": a deterministic function of the broadcast condition and the seed
    outs = torch.stack([torch.tanh(enc.sum() + ctx.sum() + torch.tensor(float(s))) for s in range(N_SONGS)])
    done = torch.zeros(N_SONGS)
    for s in mine:
        done[s] = outs[s]
    gathered = D.gather_to_rank0(done)
    m = D.max_over_ranks(float(rank) * 10)
    D.barrier()
    rec = {"rank": rank, "world": world, "local": local, "enc_sum": enc.sum().item(), "ctx_sum": ctx.sum().item(),
           "max": m, "songs": mine}
    if rank == 0:
        tot = torch.stack(gathered).sum(0)
        rec["all_songs_once"] = bool(torch.equal(tot, outs))
    with open(os.path.join(os.environ["ACEHIP_TEST_OUT"], f"rank{rank}.json"), "w") as f:
        json.dump(rec, f)
    D.destroy()


if __name__ == "__main__":
    main()
