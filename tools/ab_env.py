"""A/B of liborx builds on the learner's tick (diagnostics, round 5): for every
library given, a fresh child process times orx_env_step_ex as bench.py's
large_batch extra does (C3, int64 learner actions, RandomBot opponent,
observation / reward / done / status / refused-action count; median of 30
launches between HIP events) at 65,536 and 2^21 games, and VecEnv.step
called eagerly from a ring of two output sets (400 ticks, wall clock).
Also each size as 200 (2^21: 20) back-to-back launches between two events.
Libraries alternate over --reps rounds.

    python tools/ab_env.py lib_a.so lib_b.so [--reps=3]
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    sys.path.insert(0, ROOT)
    import ctypes
    import torch
    from bench import timed_launches
    from optimax_rogue_amd import _lib, EnvConfig
    _lib.LIB_PATH = os.path.abspath(lib.partition("@")[0])
    _lib.ABI_VERSION = ctypes.CDLL(_lib.LIB_PATH).orx_abi_version()
    from optimax_rogue_amd import VecEnv, OBS_FIELDS
    from optimax_rogue_amd.engine import BatchedEngine
    dev = torch.device("cuda", 0)
    cfg = EnvConfig.c3()
    out = {"lib": lib, "env_lanes": os.environ.get("ORX_ENV_LANES")}
    for B in (65536, 1 << 21):
        eng = BatchedEngine(cfg, B, seed=3, device=dev)
        for _ in range(2):
            eng.step(eng.policy(1, 1))
        la = torch.randint(1, 6, (B,), dtype=torch.int64, device=dev)
        lo = torch.empty((B, len(OBS_FIELDS)), dtype=torch.int32, device=dev)
        lr = torch.empty(B, dtype=torch.float32, device=dev)
        ld = torch.empty(B, dtype=torch.bool, device=dev)
        ls = torch.empty(B, dtype=torch.int32, device=dev)
        lb = torch.zeros(1, dtype=torch.int32, device=dev)
        go = lambda: eng.env_step(la, 1, lo, lr, ld, ls, lb)
        t = sorted(timed_launches(torch, go, 30))
        out[f"env_{B}"] = round(t[len(t) // 2] * 1e6, 2)
        # back to back: 200 launches between two events
        n = 200 if B <= 65536 else 20
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            go()
        b.record()
        torch.cuda.synchronize()
        out[f"env_{B}_b2b"] = round(a.elapsed_time(b) * 1e3 / n, 2)
        del eng, la, lo, lr, ld, ls, lb
        torch.cuda.empty_cache()
    # 65,536 games: 50 launches captured in one HIP graph (the device's time),
    # for int64 / int32 / int8 learner actions
    for dt in (torch.int64, torch.int32, torch.int8):
        out[f"env_65536_graph_{str(dt)[6:]}"] = graph_us(torch, cfg, dev, dt)
    pool = torch.randint(1, 6, (16, 65536), dtype=torch.int64, device=dev)
    env = VecEnv(cfg, 65536, seed=3, device=dev, opponent=1, out_buffers=2)
    for k in range(20):
        env.step(pool[k % 16])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(400):
        env.step(pool[k % 16])
    torch.cuda.synchronize()
    out["vecenv_ring_us"] = round((time.perf_counter() - t0) / 400 * 1e6, 2)
    print(json.dumps(out), flush=True)


def graph_us(torch, cfg, dev, dt):
    from optimax_rogue_amd import OBS_FIELDS
    from optimax_rogue_amd.engine import BatchedEngine
    eng = BatchedEngine(cfg, 65536, seed=3, device=dev)
    la = torch.randint(1, 6, (65536,), dtype=dt, device=dev)
    lo = torch.empty((65536, len(OBS_FIELDS)), dtype=torch.int32, device=dev)
    lr = torch.empty(65536, dtype=torch.float32, device=dev)
    ld = torch.empty(65536, dtype=torch.bool, device=dev)
    ls = torch.empty(65536, dtype=torch.int32, device=dev)
    lb = torch.zeros(1, dtype=torch.int32, device=dev)
    eng.env_step(la, 1, lo, lr, ld, ls, lb)
    g = torch.cuda.CUDAGraph()
    sg = torch.cuda.Stream(device=dev)
    sg.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(sg):
        with torch.cuda.graph(g, stream=sg):
            for _ in range(50):
                eng.env_step(la, 1, lo, lr, ld, ls, lb)
    torch.cuda.current_stream().wait_stream(sg)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(4):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1e3 / 200, 2)


def main():
    opts = dict(a[2:].split("=") for a in sys.argv[1:] if a.startswith("--") and "=" in a)
    if "--child" in sys.argv:
        return child(sys.argv[sys.argv.index("--child") + 1])
    # a library, or lib@VAR=value (the child runs with that environment
    # variable: one build, two launch settings, e.g. ORX_ENV_LANES=32)
    libs = [a for a in sys.argv[1:] if not a.startswith("--")]
    for _ in range(int(opts.get("reps", 3))):
        for spec in libs:
            lib, _, var = spec.partition("@")
            env = dict(os.environ)
            if var:
                k, v = var.split("=", 1)
                env[k] = v
            r = subprocess.run([sys.executable, __file__, "--child", spec], timeout=300, env=env)
            if r.returncode:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
