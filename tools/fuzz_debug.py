"""Diagnostics: replay one tests/test_gpu_fuzz.py case tick by tick and print
the first game-tick where the engine's rollout (one-tick launches), the
engine's policy+step and the oracle's policy+step part ways.

    python tools/fuzz_debug.py <case> [n_games_to_show]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    from oracle import oracle as oracle_lib
    from golden_util import STATE_KEYS
    from test_gpu_fuzz import _draw
    case = int(sys.argv[1])
    cfg, layouts, B, T, seed, off, pol, lanes = _draw(case)
    if lanes:
        os.environ["ORX_ROLLOUT_LANES"] = str(lanes)
    print(cfg, B, T, pol, lanes, None if layouts is None else layouts.shape)
    dev = torch.device("cuda", 0)
    ora = oracle_lib.Oracle(cfg, B, seed, off, layouts=layouts)
    ora.reset(episode=np.zeros(B, np.int32))
    mk = lambda: BatchedEngine(EnvConfig.from_dict(cfg, layouts=layouts), B, seed=seed,
                               game_offset=off, device=dev)
    er, es = mk(), mk()
    keys = [k for k in STATE_KEYS if not k.startswith("npc")] + ["p_layout", "p_rpg", "item_mask"]

    def row(s, g):
        return {k: np.asarray(s[k])[..., g].tolist() for k in keys if k in s}

    prev = (ora.export(), er.snapshot(), es.snapshot())
    for t in range(T):
        a = ora.policy(*pol)
        ora.step(a)
        er.rollout(1, *pol)
        ea = es.policy(*pol)
        es.step(ea)
        w, r, s = ora.export(), er.snapshot(), es.snapshot()
        bad = set()
        for k in keys:
            if k in w:
                for name, got in (("rollout", r), ("step", s)):
                    if k in got and not np.array_equal(np.asarray(got[k]), np.asarray(w[k])):
                        gs = np.nonzero((np.asarray(got[k]) != np.asarray(w[k])).reshape(-1, B).any(0))[0]
                        bad |= {(name, k, int(g)) for g in gs}
        if not np.array_equal(ea.cpu().numpy(), a):
            print("policy differs at t", t + 1)
        if bad:
            print("tick", t + 1, "mismatches", sorted(bad)[:10])
            for g in sorted({b[2] for b in bad})[:int(sys.argv[2]) if len(sys.argv) > 2 else 2]:
                print(" game", g, "actions", a[g].tolist())
                print("  before oracle ", row(prev[0], g))
                print("  after  oracle ", row(w, g))
                print("  after  rollout", row(r, g))
                print("  after  step   ", row(s, g))
                print("  oracle entities", ora.entities(g))
                print("  oracle world", ora.world(g))
            return
        prev = (w, r, s)
    print("no mismatch")


if __name__ == "__main__":
    main()
