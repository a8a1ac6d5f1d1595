"""Dungeon banks from 64 to 160 KiB of tiles (diagnostics, round 5): the
bench's bank workload (65,536 games on 64x64 with 8 NPCs, 2x RandomBot) on
L = 16..40 random layouts, in the launch forms the plan can take -- the
paired form with the tiles staged in LDS (256- or 512-thread workgroups),
the one-lane form with the tiles in global memory (a refused LDS raise,
forced by ORX_REFUSE_LDS_RAISE=1) -- as one and two stream shards, each timed
as the headline step (3 warmups, 20 back-to-back 128-tick steps between HIP
events, fork / join).

    python tools/bank_forms.py > bank_forms.jsonl
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
    from optimax_rogue_amd import DungeonBank, EnvConfig
    from optimax_rogue_amd.engine import StreamShardedEngine
    dev = torch.device("cuda", 0)
    T = 128
    forms = [("plan", {}), ("threads256", {"ORX_ROLLOUT_THREADS": "256"}),
             ("one_lane_global", {"ORX_REFUSE_LDS_RAISE": "1"})]
    knobs = ("ORX_ROLLOUT_THREADS", "ORX_REFUSE_LDS_RAISE")
    for rnd in range(2):
        for L in (16, 20, 24, 32, 40):
            bank = DungeonBank.random(64, 64, L, seed=7)
            cfg = EnvConfig(width=64, height=64, n_npcs=8, layouts=bank.layouts)
            for streams in (2, 1):
                for name, env in forms:
                    if name == "threads256" and L * 4096 * 2 <= 160 * 1024:
                        continue   # the plan's own choice there
                    for k in knobs:
                        os.environ.pop(k, None)
                    os.environ.update(env)
                    e = StreamShardedEngine(cfg, 65536, seed=5, device=dev, n_streams=streams)
                    o, a = e.trajectory_buffers(T)
                    go = e.rollout_launcher(T, 1, 1, obs=o, act=a)
                    us = step_us(torch, e, go)
                    print(json.dumps({"round": rnd, "layouts": L, "tiles_kib": L * 4, "form": name,
                                      "streams": streams, "shape": e.rollout_shape(1, 1),
                                      "us_per_step": round(us, 2)}), flush=True)
                    del e, o, a, go
                    torch.cuda.empty_cache()
    for k in knobs:
        os.environ.pop(k, None)


if __name__ == "__main__":
    main()
