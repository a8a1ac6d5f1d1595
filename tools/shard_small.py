"""The small per-GPU batches as stream shards (diagnostics): C2 (4,096
games) and C5's 8-GPU share (16,384 games, separation damage off and on) as
1, 2 and 4 StreamShardedEngine shards, timed as the headline step is (one
fork, back-to-back 128-tick steps on each shard's stream, one join; HIP
events around them).  A launch ends with its slowest wave; with two or more
shards one shard's next launch starts while another's tail still runs.

    python tools/shard_small.py > shard_small.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import StreamShardedEngine
    from optimax_rogue_amd.enums import EXT_SEPARATION_DAMAGE
    dev = torch.device("cuda", 0)
    c5sep = EnvConfig.c5()
    c5sep.flags, c5sep.sep_period = EXT_SEPARATION_DAMAGE, 8
    cases = [("c2", EnvConfig.c2(), 4096, 1), ("c5", EnvConfig.c5(), 16384, 2),
             ("c5sep", c5sep, 16384, 2)]
    T, reps = 128, 20
    for rnd in range(2):
        for name, cfg, games, pol in cases:
            for streams in (1, 2, 4):
                e = StreamShardedEngine(cfg, games, seed=5, device=dev, n_streams=streams)
                o, a = e.trajectory_buffers(T)
                go = e.rollout_launcher(T, pol, pol, obs=o, act=a)
                e.fork()
                for _ in range(3):
                    go()
                e.join()
                s, f = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                s.record()
                e.fork()
                for _ in range(reps):
                    go()
                e.join()
                f.record()
                torch.cuda.synchronize()
                us = s.elapsed_time(f) * 1e3 / reps
                print(json.dumps({"round": rnd, "cfg": name, "games": games, "streams": streams,
                                  "shape": e.rollout_shape(pol, pol), "us_per_step": round(us, 2),
                                  "env_steps_per_s": games * T / us * 1e6}), flush=True)
                del e, o, a, go
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
