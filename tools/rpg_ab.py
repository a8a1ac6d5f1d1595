"""C3 rollout time per launch (HIP events, median) with each character
mechanic on alone and all together, against the reference-semantics
headline form: which mechanic costs what (diagnostics).

    python tools/rpg_ab.py [games] [ticks]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from optimax_rogue_amd import EnvConfig, OBS_FIELDS
    from optimax_rogue_amd.engine import BatchedEngine
    from optimax_rogue_amd.enums import EXT_ITEMS, EXT_LEVELING, EXT_MANA, EXT_RPG
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    dev = torch.device("cuda", 0)
    obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
    act = torch.empty((T, B, 2), dtype=torch.int8, device=dev)
    variants = {"none": 0, "mana": EXT_MANA, "leveling": EXT_LEVELING, "items": EXT_ITEMS,
                "all": EXT_RPG}
    for rep in range(2):
        for name, flags in variants.items():
            e = BatchedEngine(EnvConfig(width=64, height=64, n_npcs=8, flags=flags), B, seed=5,
                              device=dev)
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
            print(json.dumps({"rep": rep, "variant": name, "flags": flags, "games": B, "ticks": T,
                              "lanes": e.rollout_lanes(), "us_per_launch": round(us, 2)}),
                  flush=True)
            del e, go


if __name__ == "__main__":
    main()
