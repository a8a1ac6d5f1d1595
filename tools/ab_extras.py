"""A/B of liborx builds over bench.py's rollout workloads (diagnostics): for
every library given, a fresh child process times, as the bench does (HIP
events; stream-shard workloads as two shards launched back to back between
one fork and one join, 3 warmup + 20 timed steps; one-stream workloads the
median of 10 launches):

  c3          the headline: C3, 65,536 games, 2x RandomBot, 2 shards
  c3_mixed    C3, RandomBot vs StaircaseBot, 2 shards
  c5_16384    C5's 8-GPU share, 2x StaircaseBot, separation damage off / on
  c5_131072   C5 on one GPU, separation damage off / on
  c2          C2: 4,096 games on 32x32, one stream
  bank        C3 on a 16-layout dungeon bank, 2 shards
  c3_rpg      C3 with the character mechanics, 2 shards

µs per 128-tick step.  Libraries alternate over --reps rounds; every line is
one library's round.

    python tools/ab_extras.py lib_a.so lib_b.so [--reps=2] [--only=c3,c5_16384]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, only):
    sys.path.insert(0, ROOT)
    import ctypes
    import torch
    from optimax_rogue_amd import _lib, EnvConfig, DungeonBank, OBS_FIELDS
    _lib.LIB_PATH = os.path.abspath(lib)
    _lib.ABI_VERSION = ctypes.CDLL(_lib.LIB_PATH).orx_abi_version()
    from optimax_rogue_amd.engine import BatchedEngine, StreamShardedEngine
    from optimax_rogue_amd.enums import EXT_RPG, EXT_SEPARATION_DAMAGE
    dev = torch.device("cuda", 0)
    T = 128

    def sharded(cfg, games, p1, p2, streams=2, reps=20):
        e = StreamShardedEngine(cfg, games, seed=5, device=dev, n_streams=streams)
        o, a = e.trajectory_buffers(T)
        go = e.rollout_launcher(T, p1, p2, obs=o, act=a)
        e.fork()
        for _ in range(3):
            go()
        e.join()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ev0.record()
        e.fork()
        for _ in range(reps):
            go()
        e.join()
        ev1.record()
        torch.cuda.synchronize()
        return round(ev0.elapsed_time(ev1) * 1e3 / reps, 2)

    def single(cfg, games, p1, p2, reps=10):
        e = BatchedEngine(cfg, games, seed=5, device=dev)
        o = torch.empty((T, len(OBS_FIELDS), games), dtype=torch.int32, device=dev)
        a = torch.empty((T, games, 2), dtype=torch.int8, device=dev)
        go = e.rollout_launcher(T, p1, p2, obs=o, act=a)
        go()
        ts = []
        for _ in range(reps):
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            go()
            ev1.record()
            torch.cuda.synchronize()
            ts.append(ev0.elapsed_time(ev1) * 1e3)
        return round(sorted(ts)[len(ts) // 2], 2)

    c5sep = EnvConfig.c5()
    c5sep.flags, c5sep.sep_period = EXT_SEPARATION_DAMAGE, 8
    work = {
        "c3": lambda: sharded(EnvConfig.c3(), 65536, 1, 1),
        "c3_mixed": lambda: sharded(EnvConfig.c3(), 65536, 1, 2),
        "c5_16384": lambda: sharded(EnvConfig.c5(), 16384, 2, 2),
        "c5_16384_sep": lambda: sharded(c5sep, 16384, 2, 2),
        "c5_131072": lambda: sharded(EnvConfig.c5(), 131072, 2, 2),
        "c5_131072_sep": lambda: sharded(c5sep, 131072, 2, 2),
        "c2": lambda: single(EnvConfig.c2(), 4096, 1, 1),
        "bank": lambda: sharded(EnvConfig(width=64, height=64, n_npcs=8,
                                          layouts=DungeonBank.random(64, 64, 16, seed=7).layouts),
                                65536, 1, 1),
        "c3_rpg": lambda: sharded(EnvConfig(width=64, height=64, n_npcs=8, flags=EXT_RPG),
                                  65536, 1, 1),
    }
    out = {"lib": lib}
    for k, fn in work.items():
        if not only or k in only:
            out[k] = fn()
            torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


def main():
    if "--child" in sys.argv:
        i = sys.argv.index("--child")
        only = sys.argv[i + 2].split(",") if len(sys.argv) > i + 2 and sys.argv[i + 2] else []
        return child(sys.argv[i + 1], only)
    opts = dict(a[2:].split("=", 1) for a in sys.argv[1:] if a.startswith("--") and "=" in a)
    libs = [a for a in sys.argv[1:] if not a.startswith("--")]
    for r in range(int(opts.get("reps", 2))):
        for lib in (libs if r % 2 == 0 else libs[::-1]):
            res = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", lib,
                                  opts.get("only", "")], capture_output=True, text=True,
                                 timeout=600)
            if res.returncode != 0:
                print(json.dumps({"lib": lib, "error": res.stderr[-800:]}), flush=True)
                return 1
            print(res.stdout.strip().splitlines()[-1], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
