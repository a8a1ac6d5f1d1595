"""In-kernel timeline of one rollout launch (diagnostics; needs a build with
-DORX_STAMPS): lane 0 of each wave records s_memtime at kernel entry (0),
after the state loads landed (1), at tick 64 (2), after the tick loop (3) and
after the epilogue's stores drained (4); per wave, the rare-block entries by
kind, the cycles spent in the rare block, its reset, ordered-tick and
descend branches, and the paired StaircaseBot form's lean ticks.

    python tools/stamps.py tools/ab_libs/stamps.so [B] [ticks]
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    lib = os.path.abspath(sys.argv[1])
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    import torch
    from optimax_rogue_amd import _lib, EnvConfig
    _lib.LIB_PATH = lib
    from optimax_rogue_amd.engine import BatchedEngine
    dev = torch.device("cuda", 0)
    # c5 / c5sep: StaircaseBot on C5's dungeon; bank: C3 on a 16-layout
    # dungeon bank; c3_rpg: C3 with the character mechanics
    cname = os.environ.get("STAMPS_CFG", "c3")
    pol = 2 if cname.startswith("c5") else 1
    pol2 = 2 if cname == "c3_mixed" else pol   # c3_mixed: RandomBot vs StaircaseBot on C3
    if cname == "bank":
        from optimax_rogue_amd import DungeonBank
        cfg = EnvConfig(width=64, height=64, n_npcs=8,
                        layouts=DungeonBank.random(64, 64, 16, seed=7).layouts)
    elif cname == "c3_rpg":
        from optimax_rogue_amd.enums import EXT_RPG
        cfg = EnvConfig(width=64, height=64, n_npcs=8, flags=EXT_RPG)
    else:
        cfg = EnvConfig.c5() if cname == "c5sep" else \
            EnvConfig.c3() if cname == "c3_mixed" else getattr(EnvConfig, cname)()
    if cname == "c5sep":
        from optimax_rogue_amd.enums import EXT_SEPARATION_DAMAGE
        cfg.flags, cfg.sep_period = EXT_SEPARATION_DAMAGE, 8
    e = BatchedEngine(cfg, B, seed=1, device=dev)
    # STAMPS_CONC: plan the launch as one of that many sharing the device (a
    # stream shard's shape, e.g. C5 131,072 as two 65,536-game shards)
    e.concurrency = int(os.environ.get("STAMPS_CONC", "1"))
    obs = torch.empty((T, 14, B), dtype=torch.int32, device=dev)
    act = torch.empty((T, B, 2), dtype=torch.int8, device=dev)
    for _ in range(4):
        e.rollout(T, pol, pol2, obs=obs, act=act)
    torch.cuda.synchronize()
    s, f = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    e.rollout(T, pol, pol2, obs=obs, act=act)
    f.record()
    torch.cuda.synchronize()
    shape = e.rollout_shape(pol, pol2)
    W = -(-B // shape["games_per_wave"])   # the launch's waves (paired: two lanes per game)
    buf = np.zeros(W * 16, dtype=np.uint64)
    dl = ctypes.CDLL(lib)
    dl.orx_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert dl.orx_diag_stamps(buf.ctypes.data, W * 16) == 0
    st = buf.reshape(W, 16)[:, :5].astype(np.int64)
    t0 = st[:, 0].min()
    st = st - t0
    # s_memtime counts the shader clock; report cycles and the event time
    out = {"B": B, "ticks": T, "cfg": cname, "games_per_wave": shape["games_per_wave"],
           "lanes_per_game": shape["lanes_per_game"], "event_us": round(s.elapsed_time(f) * 1e3, 2)}
    names = ["entry", "loaded", "tick64", "loop_end", "drained"]
    for j, n in enumerate(names):
        v = st[:, j]
        out[n] = {"min": int(v.min()), "p50": int(np.median(v)), "max": int(v.max())}
    d = np.diff(st, axis=1)
    for j, n in enumerate(["prologue", "ticks0_64", "ticks64_T", "epilogue"]):
        out["d_" + n] = {"min": int(d[:, j].min()), "p50": int(np.median(d[:, j])),
                         "max": int(d[:, j].max())}
    tot = d[:, 1] + d[:, 2]
    xcd = (np.arange(W) // 4) % 8          # 4 waves per 256-thread block, blocks round-robin
    out["loop_by_xcd_p50"] = [int(np.median(tot[xcd == x])) for x in range(8)]
    out["loop_by_xcd_max"] = [int(tot[xcd == x].max()) for x in range(8)]
    out["loop_pct"] = {q: int(np.percentile(tot, q)) for q in (1, 10, 50, 90, 99, 100)}
    rare = buf.reshape(W, 16)[:, 5:15].astype(np.int64)
    for j, n in enumerate(["rare_block", "ordered", "npc_hits", "descend", "meet", "reset"]):
        out["ticks_with_" + n] = {"mean": float(rare[:, j].mean()), "max": int(rare[:, j].max())}
    # shader-clock cycles per wave inside the rare block and three of its branches
    for j, n in enumerate(["rare_block", "reset", "ordered", "descend"]):
        v = rare[:, 6 + j]
        out["cycles_in_" + n] = {"p50": int(np.median(v)), "mean": float(v.mean())}
    lean = buf.reshape(W, 16)[:, 15].astype(np.int64)   # lean ticks (StaircaseBot spans)
    out["lean_ticks"] = {"mean": float(lean.mean()), "min": int(lean.min())}
    slow = np.argsort(tot)[-10:]
    out["slowest10_rare"] = rare[slow].tolist()
    out["slowest10_loop"] = tot[slow].tolist()
    simd = np.arange(W) % 4
    out["loop_by_wave_in_block_p50"] = [int(np.median(tot[simd == x])) for x in range(4)]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
