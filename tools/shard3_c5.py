"""C5's 8-GPU share (16,384 games, 128x128, 2x StaircaseBot) as 1, 2 and 3
stream shards, separation damage off and on, timed as the bench times its
sharded extras (diagnostics, round 5).  Two rounds.

    python tools/shard3_c5.py > shard3_c5.jsonl
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
    from optimax_rogue_amd.enums import EXT_SEPARATION_DAMAGE
    dev = torch.device("cuda", 0)
    for rnd in range(2):
        for sep in (0, 1):
            cfg = EnvConfig.c5()
            if sep:
                cfg.flags, cfg.sep_period = EXT_SEPARATION_DAMAGE, 8
            for n in (1, 2, 3):
                e = StreamShardedEngine(cfg, 16384, seed=5, device=dev, n_streams=n)
                o, a = e.trajectory_buffers(128)
                go = e.rollout_launcher(128, 2, 2, obs=o, act=a)
                print(json.dumps({"round": rnd, "sep": sep, "streams": n,
                                  "us_per_step": round(step_us(torch, e, go), 2)}), flush=True)
                del e, o, a, go
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
