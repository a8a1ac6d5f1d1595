"""What batching a wave's rare ticks could gain on C5's per-GPU share
(diagnostics, round 5; CPU only, the oracle as the trace source).

A paired wave runs its 8 games tick by tick and takes the rare block on every
tick ANY of its games needs it (a descend, a meet, a reset), so its loop is
T common ticks + U rare rounds, U the union of its games' rare ticks.  The
alternative modelled here lets a game that needs a rare tick wait (its lanes
idle, its tick counter held) until L iterations have passed, `thr` games
wait, or no game can advance without one; the rare block then serves all the
waiting games at once.  Fewer rare rounds, more loop iterations.

Traces: the oracle's C5 games (128x128, 2x StaircaseBot), 2,048 games after
512 warm-up ticks, 128 ticks recorded; a game's tick is rare when a player's
depth changes, the status leaves or is not InProgress, or the two players'
targets meet (the kernel's conditions).  Costs per wave from the stamps of
the 16,384-game launch (profiles/r04_v12/stamps_c5.json): a common tick 518
cycles (+25 for the per-lane tick bookkeeping of the lagged form), a rare
round 2,110.

    python tools/sim_rare_batching.py > profiles/r05_v13/sim_rare_batching.jsonl
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def traces(B=2048, T=128, warm=512, seed=5):
    from oracle.oracle import Oracle
    from optimax_rogue_amd import EnvConfig
    o = Oracle(EnvConfig.c5().to_dict(), B, seed)
    o.reset()
    o.rollout(2, 2, warm)
    ex = o.export()
    rare = np.zeros((T, B), bool)
    for t in range(T):
        a = o.policy(2, 2)
        o.step(a)
        nx = o.export()
        r = (nx["p_depth"] != ex["p_depth"]).any(0) | (ex["status"] != 1) | (nx["status"] != 1)
        mv = a.T
        tx = ex["p_x"] + (mv == 2) - (mv == 4)
        ty = ex["p_y"] + (mv == 3) - (mv == 1)
        same = ex["p_depth"][0] == ex["p_depth"][1]
        meet = (((tx[0] == ex["p_x"][1]) & (ty[0] == ex["p_y"][1]))
                | ((tx[1] == ex["p_x"][0]) & (ty[1] == ex["p_y"][0]))
                | ((tx[0] == tx[1]) & (ty[0] == ty[1])))
        rare[t] = r | (same & meet)
        ex = nx
    return rare


def union_cost(r, C, R):
    return r.shape[0] * C + r.any(1).sum() * R


def lagged_cost(r, L, thr, C, R):
    T, G = r.shape
    k = np.zeros(G, int)
    blocked = np.zeros(G, bool)
    wait = np.zeros(G, int)
    it = rounds = 0
    while (k < T).any():
        it += 1
        act = (k < T) & ~blocked
        nr = act & r[np.minimum(k, T - 1), np.arange(G)]
        blocked |= nr
        k[act & ~nr] += 1
        wait[blocked] += 1
        if blocked.any() and ((~blocked & (k < T)).sum() == 0 or wait[blocked].max() >= L
                              or blocked.sum() >= thr):
            rounds += 1
            k[blocked] += 1
            blocked[:] = False
            wait[:] = 0
    return it * C + rounds * R, rounds, it


def main():
    C, R, G = 518.0, 2110.0, 8
    rare = traces()
    waves = [rare[:, i:i + G] for i in range(0, rare.shape[1], G)]
    per_game = rare.sum(0)
    base = np.array([union_cost(w, C, R) for w in waves])
    print(json.dumps({"form": "union (the kernel)", "rare_ticks_per_game": float(per_game.mean()),
                      "rare_ticks_per_game_max": int(per_game.max()),
                      "rare_rounds_per_wave": float(np.mean([w.any(1).sum() for w in waves])),
                      "cycles_p50": float(np.median(base)),
                      "cycles_p99": float(np.percentile(base, 99)), "cycles_max": float(base.max())}))
    for L in (2, 4, 8, 16, 32):
        for thr in (2, 3, 4, G + 1):
            res = [lagged_cost(w, L, thr, C + 25, R) for w in waves]
            v = np.array([x[0] for x in res])
            print(json.dumps({"form": "lagged", "L": L, "thr": thr,
                              "rare_rounds_per_wave": float(np.mean([x[1] for x in res])),
                              "iterations_per_wave": float(np.mean([x[2] for x in res])),
                              "cycles_p50": float(np.median(v)),
                              "cycles_p99": float(np.percentile(v, 99)),
                              "cycles_max": float(v.max())}), flush=True)


if __name__ == "__main__":
    main()
