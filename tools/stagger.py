"""Diagnostics: the two stream shards of the bench step run in phase (both
launch 128-tick rollouts back to back) or half a launch apart (shard 1
starts and ends with a 64-tick launch) -- same ticks of work per shard.

    python tools/stagger.py [steps]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import StreamShardedEngine
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    eng = StreamShardedEngine(EnvConfig.c3(), 65536, seed=3, device=dev, n_streams=2)
    obs, act = eng.trajectory_buffers(128)
    full = [None, None]
    half = [None, None]
    for j, (e, s) in enumerate(zip(eng.parts, eng.streams)):
        with torch.cuda.stream(s):
            full[j] = e.rollout_launcher(128, 1, 1, obs=obs[j], act=act[j])
            half[j] = e.rollout_launcher(64, 1, 1, obs=obs[j][:64], act=act[j][:64])

    def run(stagger):
        eng.fork()
        if stagger:
            half[1]()
            for _ in range(K - 1):
                full[0]()
                full[1]()
            full[0]()
            half[1]()
        else:
            for _ in range(K):
                full[0]()
                full[1]()
        eng.join()

    out = {}
    for rep in range(3):
        for stagger in (False, True):
            run(stagger)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run(stagger)
            b.record()
            torch.cuda.synchronize()
            out.setdefault("stagger" if stagger else "in_phase", []).append(
                round(a.elapsed_time(b) * 1e3 / K, 2))
    print(json.dumps({"us_per_step": out, "steps": K}), flush=True)


if __name__ == "__main__":
    main()
