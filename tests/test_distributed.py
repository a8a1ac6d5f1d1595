"""CPU, world_size 2 over gloo: the sharded path (global-id game offsets and
the all-gather of episode returns) reproduces a single-process run exactly.
The per-rank stepping engine here is the oracle (the HIP engine needs a GPU;
its offset invariance is covered by tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from optimax_rogue_amd.parallel import gather_returns, shard

CFG = dict(width=7, height=6, n_npcs=2, max_ticks=40)
TICKS = 200
SEED = 17


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, global_batch, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.oracle import Oracle
    off, n = shard(global_batch, rank, world)
    o = Oracle(CFG, n, SEED, off)
    o.reset()
    o.rollout(1, 2, TICKS)
    s = o.export()
    local = torch.from_numpy(np.stack([s["ret_sum"], s["ep_count"], s["tick"]]))
    full = gather_returns(local, global_batch)
    if rank == 0:
        np.save(os.path.join(out_dir, "gathered.npy"), full.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("global_batch", [300, 301])
def test_gloo_world2_matches_single_process(tmp_path, oracle_lib, global_batch):
    mp.spawn(_worker, args=(2, _free_port(), global_batch, str(tmp_path)), nprocs=2, join=True)
    got = np.load(tmp_path / "gathered.npy")
    o = oracle_lib.Oracle(CFG, global_batch, SEED, 0)
    o.reset()
    o.rollout(1, 2, TICKS)
    s = o.export()
    want = np.stack([s["ret_sum"], s["ep_count"], s["tick"]])
    assert got.shape == want.shape
    assert np.array_equal(got, want)
    assert want[1].sum() > 0


def test_shard_partition():
    for G in (1, 7, 8, 65536 * 8 + 3):
        for W in (1, 2, 3, 8):
            spans = [shard(G, r, W) for r in range(W)]
            assert spans[0][0] == 0
            assert all(spans[r][0] + spans[r][1] == spans[r + 1][0] for r in range(W - 1))
            assert spans[-1][0] + spans[-1][1] == G
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
