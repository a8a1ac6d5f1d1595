"""Diagnostics: rollout time per launch for small batches with 256-thread
workgroups (four waves) and single-wave workgroups (ORX_ROLLOUT_THREADS).

    python tools/threads_ab.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from optimax_rogue_amd import EnvConfig, OBS_FIELDS
    from optimax_rogue_amd.engine import BatchedEngine
    dev = torch.device("cuda", 0)
    T = 128
    for rep in range(2):
        for name, cfg, B, pol in (("c2", EnvConfig.c2(), 4096, 1), ("c2_1024", EnvConfig.c2(), 1024, 1),
                                  ("c5_16384", EnvConfig.c5(), 16384, 2),
                                  ("c3_16384", EnvConfig.c3(), 16384, 1)):
            for threads in ("256", "64"):
                os.environ["ORX_ROLLOUT_THREADS"] = threads
                e = BatchedEngine(cfg, B, seed=5, device=dev)
                obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
                act = torch.empty((T, B, 2), dtype=torch.int8, device=dev)
                go = e.rollout_launcher(T, pol, pol, obs=obs, act=act)
                go()
                ts = []
                for _ in range(9):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    go()
                    b.record()
                    ts.append((a, b))
                torch.cuda.synchronize()
                us = sorted(a.elapsed_time(b) * 1e3 for a, b in ts)[4]
                print(json.dumps({"rep": rep, "case": name, "games": B, "threads": int(threads),
                                  "lanes": e.rollout_lanes(), "us_per_launch": round(us, 2),
                                  "env_steps_per_s": B * T / us * 1e6}), flush=True)
                del e, go, obs, act


if __name__ == "__main__":
    main()
