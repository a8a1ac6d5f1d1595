"""Rollout launch forms by policy pair (diagnostics, round 5): C3 (65,536
games as two stream shards, 128-tick steps timed as the headline) with both
players RandomBot, both StaircaseBot, and the mixed pairs (a RandomBot
against a StaircaseBot, either way round), with the launch shape each takes.

    python tools/mixed_forms.py > mixed_forms.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch
    from c5_forms import step_us
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import StreamShardedEngine
    dev = torch.device("cuda", 0)
    for rnd in range(2):
        for pol in ((1, 1), (2, 2), (1, 2), (2, 1)):
            e = StreamShardedEngine(EnvConfig.c3(), 65536, seed=5, device=dev, n_streams=2)
            o, a = e.trajectory_buffers(128)
            go = e.rollout_launcher(128, *pol, obs=o, act=a)
            us = step_us(torch, e, go)
            print(json.dumps({"round": rnd, "policies": pol, "shape": e.rollout_shape(*pol),
                              "us_per_step": round(us, 2)}), flush=True)
            del e, o, a, go
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
