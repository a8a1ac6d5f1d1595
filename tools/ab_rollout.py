"""A/B timing of liborx builds (diagnostics): for every library path given,
a fresh child process times the C3 headline rollout (65,536 games, 50-tick
launches with obs+act) and, with --large, 2^21 games x 20 ticks.

    python tools/ab_rollout.py optimax_rogue_amd/liborx.so /tmp/liborx_b.so \
        tools/ab_libs/diag4.so

An argument ``path@VAR=value[@...]`` runs that library with environment
variables set; ``@OBS=0`` drops the trajectory outputs.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(arg, large, ticks=50):
    lib, *envs = arg.split("@")
    with_obs = True
    abi = None
    for env in envs:
        k, _, v = env.partition("=")
        if k == "OBS":          # OBS=0: no trajectory output
            with_obs = v != "0"
        elif k == "ABI":        # ABI=n: accept an older library build (same call shapes)
            abi = int(v)
        else:
            os.environ[k] = v
    sys.path.insert(0, ROOT)
    import torch
    from optimax_rogue_amd import _lib, EnvConfig
    _lib.LIB_PATH = os.path.abspath(lib)
    if abi is not None:
        _lib.ABI_VERSION = abi
    from optimax_rogue_amd.engine import BatchedEngine
    from optimax_rogue_amd.enums import OBS_FIELDS
    dev = torch.device("cuda", 0)
    out = {"lib": arg}
    shapes = [(65536, ticks, 40, "c3", 1)] + ([(1 << 21, 20, 6, "c3", 1)] if large else [])
    if os.environ.get("AB_C5"):   # C5: 128x128 StaircaseBot at 16,384 and 131,072 games
        shapes += [(16384, 128, 20, "c5", 2), (131072, 128, 10, "c5", 2)]
    if os.environ.get("AB_SMALL"):   # batches below 64 games per wave: C2, a C3 stream shard
        shapes += [(4096, 128, 40, "c2", 1), (32768, 128, 20, "c3", 1), (16384, 128, 20, "c3", 1)]
    if os.environ.get("AB_RESETS"):  # C3 with 20-tick episodes: a reset every 20 ticks
        shapes += [(65536, 128, 20, "c3resets", 1)]
    if os.environ.get("AB_C5SEP"):   # the same with separation damage (sep_period 8)
        shapes += [(16384, 128, 20, "c5sep", 2), (131072, 128, 10, "c5sep", 2)]
    for B, T, reps, cname, pol in shapes:
        if cname == "c5sep":
            from optimax_rogue_amd.enums import EXT_SEPARATION_DAMAGE
            cfg = EnvConfig.c5()
            cfg.flags, cfg.sep_period = EXT_SEPARATION_DAMAGE, 8
        elif cname == "c3resets":
            cfg = EnvConfig.c3()
            cfg.max_ticks = 20
        else:
            cfg = getattr(EnvConfig, cname)()
        e = BatchedEngine(cfg, B, seed=1, device=dev)
        obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=dev) \
            if with_obs else None
        act = torch.empty((T, B, 2), dtype=torch.int8, device=dev) if with_obs else None
        for _ in range(3):
            e.rollout(T, pol, pol, obs=obs, act=act)
        torch.cuda.synchronize()
        s, f = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            e.rollout(T, pol, pol, obs=obs, act=act)
        f.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(f) * 1e3 / reps
        out[f"{cname}_B{B}"] = {"us_per_launch": round(us, 2), "env_steps_per_s": B * T / us * 1e6}
    print(json.dumps(out), flush=True)


def main():
    ticks = [int(a.split("=")[1]) for a in sys.argv if a.startswith("--ticks=")] or [50]
    if sys.argv[1] == "--child":
        child(sys.argv[2], "--large" in sys.argv, ticks[0])
        return
    large = "--large" in sys.argv
    for lib in [a for a in sys.argv[1:] if not a.startswith("--")]:
        for _ in range(2):
            r = subprocess.run([sys.executable, __file__, "--child", lib, f"--ticks={ticks[0]}"]
                               + (["--large"] if large else []),
                               timeout=300)
            if r.returncode:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
