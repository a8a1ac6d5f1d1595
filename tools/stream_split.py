"""C3 rollout throughput with the batch split over S HIP streams (diagnostics).

The 65,536 games are S engines of 65,536 / S games (contiguous global ids,
game_offset), each launching its 128-tick rollouts on its own stream; one
step = one launch per engine.  The launches of different streams may run
concurrently, so one part's launch tail overlaps the others' work.  Prints
env-steps/s over `steps` steps (HIP events on every stream, bracketed by
device synchronizations) for S = 1, 2, 4 and each lanes setting given.

    python tools/stream_split.py [lanes ...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from optimax_rogue_amd import EnvConfig
from optimax_rogue_amd.engine import BatchedEngine
from optimax_rogue_amd.enums import OBS_FIELDS


def run(S, B=65536, T=128, steps=20, warm=5):
    dev = torch.device("cuda", 0)
    n = B // S
    streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    engs, launch = [], []
    for k, s in enumerate(streams):
        with torch.cuda.stream(s):
            e = BatchedEngine(EnvConfig.c3(), n, seed=3, game_offset=k * n, device=dev)
            obs = torch.empty((T, len(OBS_FIELDS), n), dtype=torch.int32, device=dev)
            act = torch.empty((T, n, 2), dtype=torch.int8, device=dev)
            launch.append(e.rollout_launcher(T, 1, 1, obs=obs, act=act))
            engs.append((e, obs, act))
    torch.cuda.synchronize()
    for _ in range(warm):
        for go in launch:
            go()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        for go in launch:
            go()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"streams": S, "games_per_stream": n, "lanes": engs[0][0].rollout_lanes(),
            "us_per_step": el / steps * 1e6, "env_steps_per_s": B * T * steps / el}


def main():
    lanes = sys.argv[1:] or ["0"]
    for L in lanes:
        if L != "0":
            os.environ["ORX_ROLLOUT_LANES"] = L
        else:
            os.environ.pop("ORX_ROLLOUT_LANES", None)
        for S in (1, 2, 4):
            r = run(S)
            r["requested_lanes"] = L
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
