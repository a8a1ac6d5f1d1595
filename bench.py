#!/usr/bin/env python3
"""bench.py -- env-steps/s of the batched Optimax Rogue tick engine on MI355X.

    python bench.py [--gpus N --steps K --warmup W]          # 1 GPU
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workload (BASELINE.json configs[2], "C3"): 65,536 games per GPU on a 64x64
grid with enemies (K = 8 NPCs per game), both players driven by RandomBot,
Unreachable despawn, max_ticks 1000 with autoreset.  One "step" = one tick of
every game in the batch; an env-step = one game advanced one tick.  Games
shard across GPUs by global game id (weak scaling, no data-path collective);
after the timed region the per-game episode returns are all-gathered over
RCCL (the only collective).

Modes
  rollout (default): one fused kernel launch per --chunk ticks; state stays in
          registers and every tick's full observation (14 int32 fields) and
          actions are streamed to an HBM trajectory buffer.
  step:   per tick a policy launch then a step launch (orx_policy/orx_step),
          state read from and written back to HBM every tick.

Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
OBS_BYTES = 14 * 4      # one tick record: 14 int32 fields
ACT_BYTES = 2


def algorithmic_bytes(mode: str, K: int, ticks: int) -> dict:
    """Algorithmic HBM bytes of the dominant kernel per game per launch."""
    npc_read = (4 + 2 * K) if K else 0          # alive mask + K packed positions
    if mode == "step":
        read = 2 + 32 + 16 + 12 + npc_read        # actions, players, stairs, tick/status/episode
        write = 32 + 8                            # players, tick, status
        return {"per_unit": read + write, "per_launch_per_game": read + write, "units": 1}
    state_in = 32 + 16 + 12 + npc_read            # players, stairs, tick/status/episode, NPCs
    state_out = 32 + 12 + (4 if K else 0)         # players, tick/status/episode, alive mask
    per_tick = OBS_BYTES + ACT_BYTES
    return {"per_unit": per_tick, "per_launch_per_game": ticks * per_tick + state_in + state_out,
            "units": ticks}


def cpu_baseline(cfg_dict: dict, seconds: float) -> dict:
    """The C oracle (scalar port of the reference updater), one host core,
    same workload shape; bounded to about `seconds` of CPU work."""
    from oracle.oracle import Oracle, build
    build()
    B = 256
    ora = Oracle(cfg_dict, B, 3, 0)
    ora.reset()
    t0 = time.perf_counter()
    ticks = 0
    while True:
        ora.rollout(1, 1, 50)
        ticks += 50
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": B * ticks / el, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"C oracle (scalar C restatement of Updater.update + RandomBot), {B} games x "
                      f"{ticks} ticks of the same C3 workload on 1 host core "
                      f"({platform.processor() or platform.machine()}), {el:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000, help="ticks in the timed region")
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--batch", type=int, default=65536, help="games per GPU")
    ap.add_argument("--mode", choices=["rollout", "step"], default="rollout")
    ap.add_argument("--chunk", type=int, default=50, help="ticks per rollout launch")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from optimax_rogue_amd import EnvConfig, OBS_FIELDS
    from optimax_rogue_amd.engine import BatchedEngine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    cfg = EnvConfig.c3()
    B = args.batch
    eng = BatchedEngine(cfg, B, seed=3, game_offset=rank * B, device=dev)
    chunk = max(1, min(args.chunk, args.steps))
    obs = act = None
    if args.mode == "rollout":
        obs = torch.empty((chunk, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
        act = torch.empty((chunk, B, 2), dtype=torch.int8, device=dev)

    def run(n_ticks, events=None):
        if args.mode == "rollout":
            left = n_ticks
            while left > 0:
                t = min(chunk, left)
                if events is not None:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                eng.rollout(t, 1, 1, obs=obs, act=act)
                if events is not None:
                    e1.record()
                    events.append((e0, e1, t))
                left -= t
        else:
            for _ in range(n_ticks):
                eng.policy(1, 1)
                if events is not None:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                eng.step()
                if events is not None:
                    e1.record()
                    events.append((e0, e1, 1))

    run(args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    events = []
    t0 = time.perf_counter()
    run(args.steps, events)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # dominant kernel: average launch duration from HIP events on its stream
    durs = [a.elapsed_time(b) * 1e-3 for a, b, _ in events]
    full = [(d, n) for d, (_, _, n) in zip(durs, events) if n == chunk or args.mode == "step"]
    avg_launch_s = sum(d for d, _ in full) / max(1, len(full))
    ab = algorithmic_bytes(args.mode, cfg.n_npcs, chunk if args.mode == "rollout" else 1)
    bytes_per_launch = ab["per_launch_per_game"] * B
    achieved_gbs = bytes_per_launch / avg_launch_s / 1e9

    # the only collective: all-gather of per-game episode returns (RCCL / xGMI)
    rets = eng.episode_returns()
    gather_ms = None
    if world > 1:
        outs = [torch.empty_like(rets) for _ in range(world)]
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        dist.all_gather(outs, rets)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3
        allrets = torch.cat(outs, dim=1)
    else:
        allrets = rets
    episodes = int(allrets[1].sum().item())
    mean_ret = float(allrets[0].sum().item()) / max(1, episodes)

    total_steps = B * world * args.steps
    value = total_steps / elapsed
    result = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(cfg.to_dict(), args.cpu_seconds)
        result = {
            "metric": "env-steps/sec (whole node) at batch=65536, 64x64 grid; bit-exact vs ref",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (Philox-seeded dungeons, RandomBot actions)",
            "config": {
                "workload": "C3: 65536 games/GPU, 64x64 grid, 8 NPCs/game, 2x RandomBot, "
                            "Unreachable despawn, max_ticks 1000, autoreset",
                "batch_per_gpu": B, "global_batch": B * world, "grid": "64x64",
                "n_npcs": cfg.n_npcs, "mode": args.mode,
                "ticks_per_launch": chunk if args.mode == "rollout" else 1,
                "parallelism": f"games sharded by global id over {world} GPU(s)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "rollout_kernel" if args.mode == "rollout" else "step_kernel",
                "achieved": achieved_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS,
                "traffic": None,
                "bytes_per_launch": bytes_per_launch,
                "bytes_per_env_step": ab["per_unit"],
                "avg_launch_us": avg_launch_s * 1e6,
                "launches": len(full),
            },
            "cpu_baseline": cpu,
            "episodes_finished": episodes,
            "mean_return_p1": mean_ret,
            "returns_gather_ms": gather_ms,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
