"""Games-per-wave A/B across liborx builds (diagnostics): for each library
(path[@VAR=value...]) a fresh child process times C5 at 16,384 games and C2
at 4,096 (128-tick rollout launches with obs+act, HIP events, median of 10)
at each lanes value given.

    python tools/lanes_ab.py lib1.so lib2.so@ORX_ROLLOUT_PAIRED=0 --lanes=16,8
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(arg, lanes_list):
    lib, *envs = arg.split("@")
    for env in envs:
        k, _, v = env.partition("=")
        os.environ[k] = v
    sys.path.insert(0, ROOT)
    from optimax_rogue_amd import _lib
    _lib.LIB_PATH = os.path.abspath(lib)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from lanes_sweep import point
    from optimax_rogue_amd import EnvConfig
    work = [("c5", EnvConfig.c5(), 16384, 2), ("c2", EnvConfig.c2(), 4096, 1)]
    if os.environ.get("LANES_AB_BIG"):   # C5 on one GPU: 131,072 games
        work.append(("c5", EnvConfig.c5(), 131072, 2))
    for name, cfg, B, pol in work:
        for lanes in lanes_list:
            r = point(cfg, B, pol, lanes)
            r.update(workload=name, lib=arg)
            print(json.dumps(r), flush=True)


def main():
    lanes = [int(x) for a in sys.argv if a.startswith("--lanes=") for x in a[8:].split(",")] or [16, 8]
    if "--child" in sys.argv:
        child(sys.argv[sys.argv.index("--child") + 1], lanes)
        return
    for lib in [a for a in sys.argv[1:] if not a.startswith("--")]:
        r = subprocess.run([sys.executable, __file__, "--child", lib,
                            "--lanes=" + ",".join(map(str, lanes))], timeout=300)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
