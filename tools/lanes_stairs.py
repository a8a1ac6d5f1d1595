"""Games per wave for the StaircaseBot-bearing paired forms (diagnostics,
round 5): C3's board (65,536 games, two stream shards) with both players
StaircaseBot and with a RandomBot against a StaircaseBot, and C5's 131,072,
at 32 / 16 / 8 games per wave (ORX_ROLLOUT_LANES), timed as the headline step.

    python tools/lanes_stairs.py > lanes_stairs.jsonl
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
    cases = [("c3", EnvConfig.c3(), 65536, (2, 2)), ("c3", EnvConfig.c3(), 65536, (1, 2)),
             ("c3_nonpc", EnvConfig(width=64, height=64), 65536, (2, 2)),
             ("c5", EnvConfig.c5(), 131072, (2, 2))]
    for rnd in range(2):
        for name, cfg, B, pol in cases:
            for lanes in ("32", "16", "8"):
                os.environ["ORX_ROLLOUT_LANES"] = lanes
                e = StreamShardedEngine(cfg, B, seed=5, device=dev, n_streams=2)
                o, a = e.trajectory_buffers(128)
                go = e.rollout_launcher(128, *pol, obs=o, act=a)
                us = step_us(torch, e, go)
                print(json.dumps({"round": rnd, "cfg": name, "games": B, "policies": pol,
                                  "shape": e.rollout_shape(*pol), "us_per_step": round(us, 2)}),
                      flush=True)
                del e, o, a, go
                torch.cuda.empty_cache()
    os.environ.pop("ORX_ROLLOUT_LANES", None)


if __name__ == "__main__":
    main()
