"""Times the REFERENCE's own CPU path on this container's host cores (build
container only: /root/reference never travels to the GPU box) and writes
profiles/ref_cpu_c3.json, which bench.py reports as
cpu_baseline.reference_python.

The reference is imported read-only and unmodified -- stock CPython `random`
and `numpy.random`, nothing injected (the only stand-in is the third-party
`inflection` module it imports for serializer names, tests/golden/
make_golden.py:_underscore; nothing on the timed path calls it).  Workload =
BASELINE.json configs[2] (C3): 64x64 EmptyDungeonGenerator, Together start,
8 NPCs added after setup_game exactly as the fixtures' NpcGameStart does
(make_golden.py), DungeonDespawningStrategy.Unreachable, max_ticks 1000, both
players RandomBot; a finished game is set up again (autoreset).  One process
per core, each for `--seconds`; stdout (the reference prints in its hot path)
goes to /dev/null.  Two loops are timed:

  * updater: gs.on_tick(); Updater.update(gs, m1, m2) with actions drawn
    beforehand by RandomBot.move (the server's tick, server/main.py:110-113,
    updater.py:76-162);
  * full: RandomBot.move for both players + on_tick + update (what one
    env-step of the batched engine covers).

Beside them, on the same cores in the same run, `oracle/pyref.py` (the
pure-Python object-model restatement bench.py times on the GPU box as
`python_restatement`, where the reference cannot go): `pyref_vs_reference`
= pyref's env-steps/s / the reference's "full" leg, single core and per core
of the parallel leg, so the GPU box's python_restatement figure can be read
as the reference's cost (divide by the ratio).

    python tools/ref_cpu_baseline.py [--seconds 10] [--procs N]
"""
import argparse
import json
import multiprocessing as mp
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def _import():
    import types
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_golden import _underscore
    stub = types.ModuleType("inflection")
    stub.underscore = _underscore
    sys.modules.setdefault("inflection", stub)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import optimax_rogue.game.entities as entities
    import optimax_rogue.logic.updater as updater
    import optimax_rogue.logic.worldgen as worldgen
    import optimax_rogue_bots.randombot as randombot
    return entities, updater, worldgen, randombot


def _worker(args):
    k, seconds, mode = args
    import random
    import numpy as np
    random.seed(1000 + k)
    np.random.seed(1000 + k)
    sys.stdout = open(os.devnull, "w")
    entities, updater, worldgen, randombot = _import()
    W = H = 64
    dgen = worldgen.EmptyDungeonGenerator(W, H)
    start = worldgen.TogetherGameStartGenerator(dgen)
    upd = updater.Updater(dgen, updater.DungeonDespawningStrategy.Unreachable, 1000)
    bots = (randombot.RandomBot(1), randombot.RandomBot(2))

    def setup():
        gs = start.setup_game()
        d = gs.player_1.depth
        dung = gs.world.get_at_depth(d)
        for j in range(8):
            x, y = dung.get_random_unblocked()
            while (d, x, y) in gs.pos_lookup:
                x, y = dung.get_random_unblocked()
            gs.add_entity(entities.Entity(3 + j, d, x, y, 3, 3, 1, 0, [], dict()))
        return gs

    in_progress = updater.UpdateResult.InProgress
    gs = setup()
    steps = 0
    busy = 0.0
    t_end = time.perf_counter() + seconds
    while True:
        if mode == "updater":
            # Updater.update timed alone with pre-generated actions,
            # a fresh uniform draw over the 5 moves for each player every tick
            # (the bots' own draw, made outside the timed loop)
            acts = [(bots[0].move(gs), bots[1].move(gs)) for _ in range(64)]
            t0 = time.perf_counter()
            for m1, m2 in acts:
                gs.on_tick()
                res = upd.update(gs, m1, m2)
                steps += 1
                if res != in_progress:
                    break
            busy += time.perf_counter() - t0
        else:
            t0 = time.perf_counter()
            for _ in range(64):
                m1, m2 = bots[0].move(gs), bots[1].move(gs)
                gs.on_tick()
                res = upd.update(gs, m1, m2)
                steps += 1
                if res != in_progress:
                    break
            busy += time.perf_counter() - t0
        if res != in_progress:
            gs = setup()
        if time.perf_counter() >= t_end:
            break
    return steps, busy


def _cpu_model():
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--procs", type=int, default=os.cpu_count())
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "ref_cpu_c3.json"))
    a = ap.parse_args()
    import numpy
    out = {"_source": "tools/ref_cpu_baseline.py: the reference's own updater (imported "
                      "read-only from /root/reference, stock random/numpy) timed in the build "
                      "container; the reference cannot run on the GPU box",
           "workload": "C3: 64x64 EmptyDungeonGenerator, Together start, 8 NPCs, Unreachable, "
                       "max_ticks 1000, 2x RandomBot, autoreset",
           "host": _cpu_model(), "cpus": os.cpu_count(), "python": platform.python_version(),
           "numpy": numpy.__version__}
    for mode in ("updater", "full"):
        with mp.get_context("spawn").Pool(1) as p:
            s1, b1 = p.map(_worker, [(0, a.seconds, mode)])[0]
        with mp.get_context("spawn").Pool(a.procs) as p:
            t0 = time.perf_counter()
            res = p.map(_worker, [(k, a.seconds, mode) for k in range(a.procs)])
            wall = time.perf_counter() - t0
        steps = sum(s for s, _ in res)
        out[mode] = {"single_core_env_steps_per_s": s1 / b1, "procs": a.procs,
                     "aggregate_env_steps_per_s": sum(s / b for s, b in res),
                     "per_core_env_steps_per_s": sum(s / b for s, b in res) / a.procs,
                     "env_steps": steps, "seconds_per_proc": a.seconds,
                     "wall_s": wall}
    # the restatement on the same host: one core, then a.procs processes
    sys.path.insert(0, ROOT)
    from oracle import pyref
    pr = pyref.bench(a.seconds, a.procs, a.seconds)
    full = out["full"]
    out["pyref"] = {k: pr[k] for k in ("single_core", "per_core", "value", "cores", "sample")}
    out["pyref_vs_reference"] = {
        "single_core": pr["single_core"] / full["single_core_env_steps_per_s"],
        "per_core": pr["per_core"] / full["per_core_env_steps_per_s"],
        "note": "oracle/pyref.py env-steps/s over the reference's 'full' leg on this host: "
                "python_restatement (GPU box) / this ratio = the reference's own rate there"}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
