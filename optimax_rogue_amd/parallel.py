"""Multi-GPU layer: one process per GPU, games sharded by global id.

Games are independent, so there is no data-path collective: rank r owns the
contiguous global game ids ``[offset, offset + count)`` and passes ``offset``
as the engine's ``game_offset`` (the Philox counter uses the global id, so a
game's trajectory is the same for any GPU count).  The only collective is
``gather_returns``: an all-gather of the per-game episode returns after a
measurement window (``torch.distributed``: RCCL over xGMI on ROCm GPUs, gloo on
CPU).  The reference has no counterpart (it runs one game per OS process,
readme.md:59-60).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def shard(global_batch: int, rank: int, world: int) -> Tuple[int, int]:
    """(offset, count) of rank's contiguous slice; sizes differ by at most 1."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(int(global_batch), world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def env_rank() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: Optional[str] = None, device: Optional[torch.device] = None,
         force: bool = False) -> Tuple[int, int]:
    """Initializes the default process group if WORLD_SIZE > 1, or with
    ``force`` for any world size (nccl = RCCL for GPU tensors, bound to
    ``device``; gloo otherwise).  Returns (rank, world)."""
    rank, world, _ = env_rank()
    if (world > 1 or force) and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if device is not None and device.type == "cuda" else "gloo"
        kw = {"device_id": device} if backend == "nccl" and device is not None else {}
        dist.init_process_group(backend, **kw)
    return rank, world


def gather_returns(local: torch.Tensor, global_batch: int,
                   group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """All-gathers ``local`` [F, count_r] (e.g. ret_sum / ep_count rows) from every
    rank into [F, global_batch] in global game id order.  Shards may differ in
    size by one game; they are padded to a common width for the collective."""
    if not dist.is_initialized():
        return local
    world = dist.get_world_size(group)
    width = -(-int(global_batch) // world)
    # gloo collectives run on host tensors; nccl (RCCL) on device tensors
    dev = local.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    padded = torch.zeros((local.shape[0], width), dtype=local.dtype, device=dev)
    padded[:, : local.shape[1]] = local.to(dev)
    outs = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(outs, padded, group=group)
    parts = [outs[r][:, : shard(global_batch, r, world)[1]] for r in range(world)]
    return torch.cat(parts, dim=1).to(local.device)
