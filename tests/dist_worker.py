"""One rank of the sharded HIP engine, run under torchrun by
tests/test_gpu_distributed.py (every rank on cuda:0 of a 1-GPU box, gloo).

Rank r of W owns global games parallel.shard(G, r, W), steps them with its
own BatchedEngine at that game_offset, and the per-game rows are
all-gathered with parallel.gather_returns (the bench's only collective);
rank 0 writes them to --out."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from optimax_rogue_amd import EnvConfig  # noqa: E402
from optimax_rogue_amd.engine import BatchedEngine  # noqa: E402
from optimax_rogue_amd.parallel import env_rank, gather_returns, init, shard  # noqa: E402

ROWS = ("ret_sum", "ep_count", "tick", "status", "episode")


def rows_of(eng):
    """Per-game int32 rows [F, n]: returns, episode counts, tick, status,
    episode, then both players' x, y, depth, health."""
    r = [getattr(eng, k) for k in ROWS]
    for f in ("p_x", "p_y", "p_depth", "p_health"):
        r += [getattr(eng, f)[0], getattr(eng, f)[1]]
    return torch.stack(r)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--global-batch", type=int, required=True)
    ap.add_argument("--ticks", type=int, required=True)
    ap.add_argument("--cfg", required=True)
    ap.add_argument("--policy", default="1,2")
    ap.add_argument("--seed", type=int, default=23)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    rank, world, _ = env_rank()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    init("gloo", dev)
    off, n = shard(a.global_batch, rank, world)
    eng = BatchedEngine(EnvConfig.from_dict(json.loads(a.cfg)), n, seed=a.seed, game_offset=off,
                        device=dev)
    p1, p2 = (int(x) for x in a.policy.split(","))
    eng.rollout(a.ticks, p1, p2)
    full = gather_returns(rows_of(eng), a.global_batch)
    if rank == 0:
        np.save(a.out, full.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
