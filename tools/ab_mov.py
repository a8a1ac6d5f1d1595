"""A/B of the moving-NPC rollout (mov_rollout_kernel) over games per wave
(env ORX_MOV_LANES, read per launch): bench.py's c3_moving_npcs /
c3_chasing_npcs shape (C3 with npc_policy RANDOM / CHASE, 65,536 games,
2x RandomBot, 128 ticks, int32 rows + actions), median of 10 launches between
HIP events per form; every form's rows and final state are checked equal to
the first form's.  Prints one JSON line per policy and round.

    python tools/ab_mov.py [rounds] [lanes,...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    forms = sys.argv[2].split(",") if len(sys.argv) > 2 else ["64", "32", "16"]
    import torch
    from optimax_rogue_amd import EnvConfig, NpcPolicy, OBS_FIELDS, Policy
    from optimax_rogue_amd.engine import BatchedEngine
    dev = torch.device("cuda", 0)
    B, T, reps = 65536, 128, 10

    def run(cfg, lanes):
        os.environ["ORX_MOV_LANES"] = lanes
        try:
            eng = BatchedEngine(cfg, B, seed=3, device=dev)
            obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
            act = torch.empty((T, B, 2), dtype=torch.int8, device=dev)
            eng.rollout(T, Policy.Random, Policy.Random, obs=obs, act=act)
            torch.cuda.synchronize()
            first = (obs.cpu(), act.cpu(), eng.snapshot())
            ts = []
            for _ in range(reps):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                eng.rollout(T, Policy.Random, Policy.Random, obs=obs, act=act)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            return sorted(ts)[len(ts) // 2], first
        finally:
            del os.environ["ORX_MOV_LANES"]

    for r in range(rounds):
        for name, pol in (("random", NpcPolicy.Random), ("chase", NpcPolicy.Chase)):
            cfg = EnvConfig(64, 64, n_npcs=8, npc_policy=int(pol))
            out = {"round": r, "npc_policy": name}
            base = None
            for lanes in forms:
                us, res = run(cfg, lanes)
                out[f"lanes{lanes}_us"] = us
                if base is None:
                    base = res
                else:
                    same = torch.equal(res[0], base[0]) and torch.equal(res[1], base[1]) and all(
                        (res[2][k] == base[2][k]).all() for k in base[2])
                    out[f"lanes{lanes}_equal"] = bool(same)
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
