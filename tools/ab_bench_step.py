"""A/B of the bench's own step across liborx builds (diagnostics): for every
library path given, a fresh child process times the headline step -- C3,
65,536 games as two stream shards, one 128-tick rollout launch per shard with
obs+act -- over `steps` steps after `warmup`, like bench.py (HIP events, the
shards joined on the caller's stream).  Libraries alternate, `reps` rounds.

    python tools/ab_bench_step.py old.so new.so[@VAR=value...] [--reps=3] [--steps=20]

(``@STREAMS=n`` sets the shard count; other ``@VAR=value`` set environment
variables, e.g. ``@ORX_PC=1``.)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(arg, steps, warmup=5, T=128, B=65536):
    lib, *envs = arg.split("@")   # path@VAR=value: run that library with VAR set
    streams = 2
    for env in envs:
        k, _, v = env.partition("=")
        if k == "STREAMS":
            streams = int(v)
        else:
            os.environ[k] = v
    sys.path.insert(0, ROOT)
    import ctypes
    import torch
    from optimax_rogue_amd import _lib, EnvConfig
    _lib.LIB_PATH = os.path.abspath(lib)
    # an older build (another ABI) runs too: this step calls only entry
    # points whose signatures every ABI since 4 shares
    _lib.ABI_VERSION = ctypes.CDLL(_lib.LIB_PATH).orx_abi_version()
    from optimax_rogue_amd.engine import StreamShardedEngine
    dev = torch.device("cuda", 0)
    eng = StreamShardedEngine(EnvConfig.c3(), B, seed=0, device=dev,
                              n_streams=streams)
    obs, act = eng.trajectory_buffers(T)
    go = eng.rollout_launcher(T, 1, 1, obs=obs, act=act)
    eng.fork()
    for _ in range(warmup):
        go()
    eng.join()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    eng.fork()
    for _ in range(steps):
        go()
    eng.join()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / steps
    print(json.dumps({"lib": arg, "us_per_step": round(us, 2),
                      "env_steps_per_s": B * T / us * 1e6}), flush=True)


def main():
    opts = dict(a[2:].split("=") for a in sys.argv[1:] if a.startswith("--") and "=" in a)
    if "--child" in sys.argv:
        child(sys.argv[sys.argv.index("--child") + 1], int(opts.get("steps", 20)))
        return
    libs = [a for a in sys.argv[1:] if not a.startswith("--")]
    for _ in range(int(opts.get("reps", 3))):
        for lib in libs:
            r = subprocess.run([sys.executable, __file__, "--child", lib,
                                f"--steps={opts.get('steps', 20)}"], timeout=300)
            if r.returncode:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
