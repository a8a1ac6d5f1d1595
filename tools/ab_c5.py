"""A/B of liborx builds on C5 (diagnostics, round 5): for every library
given, a fresh child process times C5 as the bench does -- 16,384 games (the
8-GPU share) and 131,072 (one GPU) as two stream shards, separation damage
off and on -- each as the headline step is timed.  Libraries alternate over
--reps rounds.

    python tools/ab_c5.py lib_a.so lib_b.so [--reps=3]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import ctypes
    import torch
    from c5_forms import step_us
    from optimax_rogue_amd import _lib, EnvConfig
    _lib.LIB_PATH = os.path.abspath(lib)
    _lib.ABI_VERSION = ctypes.CDLL(_lib.LIB_PATH).orx_abi_version()
    from optimax_rogue_amd.engine import StreamShardedEngine
    from optimax_rogue_amd.enums import EXT_SEPARATION_DAMAGE
    dev = torch.device("cuda", 0)
    out = {"lib": lib}
    for sep in (0, 1):
        cfg = EnvConfig.c5()
        if sep:
            cfg.flags, cfg.sep_period = EXT_SEPARATION_DAMAGE, 8
        for B in (16384, 131072):
            e = StreamShardedEngine(cfg, B, seed=5, device=dev, n_streams=2)
            o, a = e.trajectory_buffers(128)
            go = e.rollout_launcher(128, 2, 2, obs=o, act=a)
            out[f"sep{sep}_{B}"] = round(step_us(torch, e, go), 2)
            del e, o, a, go
            torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


def main():
    opts = dict(a[2:].split("=") for a in sys.argv[1:] if a.startswith("--") and "=" in a)
    if "--child" in sys.argv:
        return child(sys.argv[sys.argv.index("--child") + 1])
    libs = [a for a in sys.argv[1:] if not a.startswith("--")]
    for _ in range(int(opts.get("reps", 3))):
        for lib in libs:
            r = subprocess.run([sys.executable, __file__, "--child", lib], timeout=300)
            if r.returncode:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
