"""C3 rollout time per launch (HIP events, median) against the NPC count:
register slots (K <= 16) and the dense occupancy-grid form (K > 16)
(diagnostics).

    python tools/npc_ab.py [games] [ticks]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from optimax_rogue_amd import EnvConfig, OBS_FIELDS
    from optimax_rogue_amd.engine import BatchedEngine
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    dev = torch.device("cuda", 0)
    obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
    act = torch.empty((T, B, 2), dtype=torch.int8, device=dev)
    for K in (8, 16, 17, 32, 64, 128, 255):
        e = BatchedEngine(EnvConfig(width=64, height=64, n_npcs=K), B, seed=5, device=dev)
        go = e.rollout_launcher(T, 1, 1, obs=obs, act=act)
        go()
        ts = []
        for _ in range(8):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            go()
            b.record()
            ts.append((a, b))
        torch.cuda.synchronize()
        us = sorted(a.elapsed_time(b) * 1e3 for a, b in ts)[4]
        print(json.dumps({"npcs": K, "form": "dense grid" if K > 16 else "registers",
                          "games": B, "ticks": T, "lanes": e.rollout_lanes(),
                          "us_per_launch": round(us, 2), "env_steps_per_s": B * T / us * 1e6}),
              flush=True)
        del e, go


if __name__ == "__main__":
    main()
