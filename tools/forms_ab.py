"""Paired vs one-lane rollout forms for the character mechanics (PM 3) and a
dungeon bank (diagnostics): µs per 128-tick step at several batches, as one
engine or as two stream shards (the headline's layout), with the paired form
allowed (default) or not (ORX_ROLLOUT_PAIRED=0, read per launch), and for
two shards also the paired form forced to 32 games per wave
(ORX_ROLLOUT_LANES=32: the plan's own rule may decline it).  Every variant is
timed twice, the second pass in reverse order.

    python tools/forms_ab.py > forms.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from optimax_rogue_amd import DungeonBank, EnvConfig
    from optimax_rogue_amd.engine import StreamShardedEngine
    from optimax_rogue_amd.enums import EXT_RPG
    dev = torch.device("cuda", 0)
    bank = DungeonBank.random(64, 64, 16, seed=7)
    cfgs = {"c3_rpg": EnvConfig(width=64, height=64, n_npcs=8, flags=EXT_RPG),
            "bank": EnvConfig(width=64, height=64, n_npcs=8, layouts=bank.layouts),
            "c3": EnvConfig.c3()}
    T, reps = 128, 8
    for name, cfg in cfgs.items():
        for games, streams in ((65536, 1), (65536, 2), (16384, 1), (4096, 1)):
            variants = [("1", ""), ("0", "")] + ([("1", "32")] if streams == 2 else [])
            # two passes, the second in reverse order: an order effect (clock
            # ramp, first use of a kernel) shows as a pass-to-pass difference
            for pas, (paired, lanes) in [(0, v) for v in variants] + [(1, v) for v in variants[::-1]]:
                os.environ["ORX_ROLLOUT_PAIRED"] = paired
                if lanes:
                    os.environ["ORX_ROLLOUT_LANES"] = lanes
                else:
                    os.environ.pop("ORX_ROLLOUT_LANES", None)
                e = StreamShardedEngine(cfg, games, seed=5, device=dev, n_streams=streams)
                o, a = e.trajectory_buffers(T)
                go = e.rollout_launcher(T, 1, 1, obs=o, act=a)
                e.fork()
                for _ in range(2):
                    go()
                e.join()
                s, f = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                s.record()
                e.fork()
                for _ in range(reps):
                    go()
                e.join()
                f.record()
                torch.cuda.synchronize()
                us = s.elapsed_time(f) * 1e3 / reps
                sh = e.rollout_shape(1, 1)
                print(json.dumps({"cfg": name, "games": games, "streams": streams, "pass": pas,
                                  "paired_allowed": paired == "1", "lanes_forced": lanes or None,
                                  "shape": sh,
                                  "us_per_step": round(us, 2),
                                  "env_steps_per_s": games * T / us * 1e6}), flush=True)
                del e, o, a, go
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
