"""Build-container check (imports /root/reference, like make_golden.py; never
run on the GPU box): the reference itself against the C oracle on the seeded
random configurations of tests/test_gpu_fuzz.py -- the ones inside the
reference's semantics (no extension flag; RandomBot / StaircaseBot players;
the players' own attributes at the reference's hard-coded 10 / 2 / 1).

For each such configuration, make_golden.run_case drives the unmodified
reference updater and bots over a few games (the configuration's own seed,
game offset, ticks, dungeon bank and stream mode) into a temporary fixture,
and tests/test_oracle.py's fixture check replays it on the oracle: state,
World.dungeons, update events and entity order every tick.  Together with the
GPU sweep (engine vs oracle on the same draws) this closes reference ->
oracle -> engine over configurations no hand-written case names.

    python tests/golden/sweep_reference.py [n_cases] [base] > profiles/ref_sweep.jsonl
"""
import contextlib
import io
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
sys.path[:0] = [HERE, TESTS, os.path.dirname(TESTS)]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    base = sys.argv[2] if len(sys.argv) > 2 else "1000"
    os.environ["ORX_FUZZ_BASE"] = base
    import golden_util
    import make_golden as MG
    import test_gpu_fuzz as F
    import test_oracle
    from oracle import oracle as oracle_lib
    oracle_lib.build()
    R = MG.import_reference()
    tmp = tempfile.mkdtemp(prefix="orx_ref_sweep_")
    MG.HERE = golden_util.GOLDEN_DIR = tmp
    n_ok = n_skip = 0
    for case in range(n):
        cfg, layouts, B, T, seed, off, pol, lanes = F._draw(case)
        if cfg["flags"] or 3 in pol:
            n_skip += 1
            continue
        # the reference's players are Entity(..., 10, 10, 2, 1, ...)
        # (worldgen.py:85-86); the NPC attributes are the spawner's
        cfg = dict(cfg, player_health=10, player_damage=2, player_armor=1)
        name = f"sweep_{base}_{case}"
        spec = dict(cfg=dict(cfg, policy=pol, layouts=layouts), seed=seed, games=min(B, 6),
                    ticks=T, offset=off)
        t0 = time.time()
        log = io.StringIO()
        with contextlib.redirect_stdout(log):
            MG.run_case(R, name, spec)
        test_oracle.test_oracle_vs_reference_fixture(oracle_lib, name)   # raises on mismatch
        os.remove(os.path.join(tmp, name + ".npz"))
        n_ok += 1
        print(json.dumps({"case": case, "base": int(base), "cfg": cfg, "bank": layouts is not None,
                          "games": min(B, 6), "ticks": T, "policy": pol, "oracle_matches": True,
                          "reference": log.getvalue().strip().split(": ", 1)[-1],
                          "s": round(time.time() - t0, 2)}), flush=True)
    print(json.dumps({"summary": {"checked": n_ok, "skipped_extension_or_stay": n_skip,
                                  "base": int(base)}}), flush=True)


if __name__ == "__main__":
    main()
