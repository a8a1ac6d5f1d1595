"""A/B of liborx builds on orx_step_n (diagnostics, round 5): for every
library given, a fresh child process replays a 128-tick move log (int8
[128, B, 2], uniform 1..5) over C3's 65,536 games as bench.py's
replay_step_n extra does (median of 10 launches between HIP events), with
int32 rows, compact rows and no rows.  Libraries alternate over --reps rounds;
--forms also times each library with ORX_STEP_N_GENERIC=1 (the generic
one-lane tick instead of the fast replay form); --lanes=32,64 times each
games-per-wave override (ORX_ROLLOUT_LANES) in turn.

    python tools/ab_replay.py lib_a.so lib_b.so [--reps=3] [--forms] [--lanes=32,64]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    sys.path.insert(0, ROOT)
    import ctypes
    import torch
    from bench import timed_launches
    from optimax_rogue_amd import _lib, EnvConfig
    _lib.LIB_PATH = os.path.abspath(lib)
    _lib.ABI_VERSION = ctypes.CDLL(_lib.LIB_PATH).orx_abi_version()
    from optimax_rogue_amd.engine import BatchedEngine, obs_rows
    from optimax_rogue_amd.enums import OBS_COMPACT, OBS_INT32
    dev = torch.device("cuda", 0)
    B, T = 65536, 128
    out = {"lib": lib, "generic_env": os.environ.get("ORX_STEP_N_GENERIC", "0"),
           "lanes_env": os.environ.get("ORX_ROLLOUT_LANES", "")}
    eng = BatchedEngine(EnvConfig.c3(), B, seed=3, device=dev)
    log = torch.randint(1, 6, (T, B, 2), dtype=torch.int8, device=dev)
    for name, fmt in (("int32", OBS_INT32), ("compact", OBS_COMPACT), ("none", None)):
        obs = None if fmt is None else torch.empty((T, obs_rows(fmt), B), dtype=torch.int32,
                                                   device=dev)
        go = (lambda: eng.step_n(log)) if obs is None else \
            (lambda: eng.step_n(log, obs=obs, obs_format=fmt))
        go()
        t = sorted(timed_launches(torch, go, 10))
        out[name] = round(t[len(t) // 2] * 1e6, 2)
    print(json.dumps(out), flush=True)


def main():
    opts = dict(a[2:].split("=") for a in sys.argv[1:] if a.startswith("--") and "=" in a)
    if "--child" in sys.argv:
        return child(sys.argv[sys.argv.index("--child") + 1])
    libs = [a for a in sys.argv[1:] if not a.startswith("--")]
    envs = ("0", "1") if "--forms" in sys.argv else ("0",)
    lanes = opts["lanes"].split(",") if "lanes" in opts else [""]
    for _ in range(int(opts.get("reps", 3))):
        for lib in libs:
            for g in envs:
                for ln in lanes:
                    env = dict(os.environ, ORX_STEP_N_GENERIC=g)
                    if ln:
                        env["ORX_ROLLOUT_LANES"] = ln
                    r = subprocess.run([sys.executable, __file__, "--child", lib], timeout=300,
                                       env=env)
                    if r.returncode:
                        sys.exit(r.returncode)


if __name__ == "__main__":
    main()
