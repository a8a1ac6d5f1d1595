"""Where the moving-NPC rollout's cycles go (diagnostics; needs a build with
-DORX_STAMPS, `python -m optimax_rogue_amd.build --variant stamps`): one
mov_rollout_kernel launch at bench.py's c3_moving_npcs / c3_chasing_npcs
shape (C3 with npc_policy RANDOM / CHASE, 65,536 games, 2x RandomBot, 128
ticks, int32 rows + actions); per wave, the shader-clock cycles of each
section summed over the launch by the wave's first active lane (slots of
ORX_MCYC_* in orx_engine.hip).  Prints the median and 90th percentile per
section over the waves, and the share of the loop.

    python tools/stamps_mov.py tools/ab_libs/stamps.so [B] [ticks]
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SECTIONS = {0: "prep (targets, initiative, NPC depth)", 1: "decide_npc_move x K",
            2: "NPC shuffle", 3: "players' handle_move", 4: "NPCs' handle_move",
            5: "end_tick", 6: "policy + tick block", 7: "autoreset", 8: "trajectory row",
            9: "tick loop", 10: "tick_moving"}


def main():
    lib = os.path.abspath(sys.argv[1])
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    import torch
    from optimax_rogue_amd import _lib, EnvConfig, NpcPolicy, OBS_FIELDS, Policy
    _lib.LIB_PATH = lib
    from optimax_rogue_amd.engine import BatchedEngine
    dev = torch.device("cuda", 0)
    L = _lib.load()
    L.orx_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    n_waves = (B + 63) // 64
    for name, pol in (("random", NpcPolicy.Random), ("chase", NpcPolicy.Chase)):
        cfg = EnvConfig(64, 64, n_npcs=8, npc_policy=int(pol))
        eng = BatchedEngine(cfg, B, seed=3, device=dev)
        obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
        act = torch.empty((T, B, 2), dtype=torch.int8, device=dev)
        eng.rollout(T, Policy.Random, Policy.Random, obs=obs, act=act)   # warm
        torch.cuda.synchronize()
        assert L.orx_diag_stamps_clear() == 0
        eng.rollout(T, Policy.Random, Policy.Random, obs=obs, act=act)
        torch.cuda.synchronize()
        buf = np.zeros(n_waves * 16, np.uint64)
        assert L.orx_diag_stamps(buf.ctypes.data, buf.size) == 0
        st = buf.reshape(n_waves, 16).astype(np.float64)
        loop = st[:, 9]
        out = {"npc_policy": name, "games": B, "ticks": T, "waves": n_waves,
               "loop_cycles_p50": float(np.median(loop)),
               "per_tick_cycles_p50": float(np.median(loop)) / T, "sections": {}}
        for j, label in SECTIONS.items():
            v = st[:, j]
            out["sections"][label] = {"p50": float(np.median(v)),
                                      "p90": float(np.percentile(v, 90)),
                                      "share_of_loop": float(np.median(v / np.maximum(loop, 1)))}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
