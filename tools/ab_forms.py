"""A/B of liborx builds on the bench's paired RandomBot forms (diagnostics,
round 5): for every library given, a fresh child process times the headline
step in compact rows (ORX_OBS_COMPACT) and in int32 rows (C3, 65,536 games as
two stream shards) and C2 (4,096 games, one launch), each as the headline
step is timed (3 warmups, 20 back-to-back 128-tick steps between HIP
events).  Libraries alternate over --reps rounds.

    python tools/ab_forms.py lib_a.so lib_b.so [--reps=3]
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
    from optimax_rogue_amd.enums import OBS_COMPACT, OBS_INT32
    dev = torch.device("cuda", 0)
    out = {"lib": lib}
    for name, cfg, B, streams, fmt in (("compact", EnvConfig.c3(), 65536, 2, OBS_COMPACT),
                                       ("int32", EnvConfig.c3(), 65536, 2, OBS_INT32),
                                       ("c2", EnvConfig.c2(), 4096, 1, OBS_INT32)):
        e = StreamShardedEngine(cfg, B, seed=3, device=dev, n_streams=streams)
        o, a = e.trajectory_buffers(128, fmt)
        go = e.rollout_launcher(128, 1, 1, obs=o, act=a, obs_format=fmt)
        out[name] = round(step_us(torch, e, go), 2)
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
