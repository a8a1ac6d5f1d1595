"""Rollout throughput vs batch size at a fixed tick range (diagnostics):
every batch starts fresh (reset), runs `warm` ticks, then times `reps`
launches of T ticks with obs+act."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from optimax_rogue_amd import EnvConfig
from optimax_rogue_amd.engine import BatchedEngine
from optimax_rogue_amd.enums import OBS_FIELDS


def run(B, T=20, warm=40, reps=5, with_obs=True, cfg=None):
    dev = torch.device("cuda", 0)
    e = BatchedEngine(cfg or EnvConfig.c3(), B, seed=1, device=dev)
    obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=dev) if with_obs else None
    act = torch.empty((T, B, 2), dtype=torch.int8, device=dev) if with_obs else None
    e.rollout(warm, 1, 1)
    torch.cuda.synchronize()
    s, f = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        e.rollout(T, 1, 1, obs=obs, act=act)
    f.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(f) * 1e3 / reps
    return us, B * T / us * 1e6


def main():
    if "--ticks" in sys.argv:   # per-launch intercept vs per-tick slope at the config batch
        for T in (10, 25, 50, 100, 200):
            us, v = run(65536, T=T, warm=200, reps=10)
            print(json.dumps({"B": 65536, "T": T, "us": round(us, 2),
                              "steps_per_s": f"{v:.3e}"}), flush=True)
        return
    for B in (65536, 131072, 262144, 524288, 1 << 20, 1 << 21):
        for obs in (True, False):
            us, v = run(B, with_obs=obs)
            print(json.dumps({"B": B, "obs": obs, "us": round(us, 1), "steps_per_s": f"{v:.3e}",
                              "ps_per_game_tick": round(us * 1e6 / (B * 20), 2)}), flush=True)
    # late tick range (resets happen): 65536 games after 2000 ticks
    dev = torch.device("cuda", 0)
    for warm in (40, 2000):
        us, v = run(65536, T=50, warm=warm, reps=20)
        print(json.dumps({"B": 65536, "warm": warm, "T": 50, "us": round(us, 1),
                          "steps_per_s": f"{v:.3e}"}), flush=True)


if __name__ == "__main__":
    main()
