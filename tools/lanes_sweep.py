"""Games-per-wave sweep of the fused rollout (diagnostics, one GPU).

For each workload and each lanes value (ORX_ROLLOUT_LANES, read by liborx
per launch) a fresh engine runs `warm` launches, then `reps` timed launches
of T ticks with obs+act; prints one JSON line per point: HIP-event us per
launch (median) and env-steps/s.

    python tools/lanes_sweep.py [c3|c5|c2|c5sep|large ...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from optimax_rogue_amd import EnvConfig
from optimax_rogue_amd.engine import BatchedEngine
from optimax_rogue_amd.enums import EXT_SEPARATION_DAMAGE, OBS_FIELDS


def point(cfg, B, pol, lanes, T=128, warm=3, reps=10):
    if lanes:
        os.environ["ORX_ROLLOUT_LANES"] = str(lanes)
    else:
        os.environ.pop("ORX_ROLLOUT_LANES", None)
    dev = torch.device("cuda", 0)
    e = BatchedEngine(cfg, B, seed=5, device=dev)
    obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
    act = torch.empty((T, B, 2), dtype=torch.int8, device=dev)
    go = e.rollout_launcher(T, pol, pol, obs=obs, act=act)
    for _ in range(warm):
        go()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    torch.cuda.synchronize()
    for a, b in ev:
        a.record()
        go()
        b.record()
    torch.cuda.synchronize()
    d = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    us = d[len(d) // 2]
    return {"games": B, "lanes": e.rollout_lanes(), "us_per_launch": round(us, 2),
            "env_steps_per_s": B * T / us * 1e6}


def bank_cfg():
    """C3 on a dungeon bank: 16 random 64x64 layouts, K = 8, RandomBots."""
    from optimax_rogue_amd import DungeonBank
    bank = DungeonBank.random(64, 64, 16, seed=7)
    return EnvConfig(width=64, height=64, n_npcs=8, layouts=bank.layouts)


def main():
    which = sys.argv[1:] or ["c3", "c5", "c2"]
    c5sep = EnvConfig.c5()
    c5sep.flags, c5sep.sep_period = EXT_SEPARATION_DAMAGE, 8
    work = {"c3": [(EnvConfig.c3(), 65536, 1)],
            "c5": [(EnvConfig.c5(), 16384, 2), (EnvConfig.c5(), 131072, 2)],
            "c5sep": [(c5sep, 16384, 2), (c5sep, 131072, 2)],
            "c2": [(EnvConfig.c2(), 4096, 1)],
            "large": [(EnvConfig.c3(), 1 << 20, 1)],
            "bank": [(bank_cfg(), 65536, 1), (bank_cfg(), 16384, 1)]}
    for w in which:
        for cfg, B, pol in work[w]:
            if w == "bank":  # LDS-staged tiles against L2-resident global reads
                for no_lds in ("", "1"):
                    if no_lds:
                        os.environ["ORX_NO_LDS_TILES"] = "1"
                    else:
                        os.environ.pop("ORX_NO_LDS_TILES", None)
                    r = point(cfg, B, pol, 0)
                    r.update(workload=w, lds_tiles=not no_lds)
                    print(json.dumps(r), flush=True)
                os.environ.pop("ORX_NO_LDS_TILES", None)
                continue
            for lanes in (0, 64, 32, 16, 8, 4, 2):
                if lanes and B // lanes > (1 << 16):
                    continue
                r = point(cfg, B, pol, lanes)
                r.update(workload=w, requested=lanes or "default")
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
