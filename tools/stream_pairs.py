"""Does a two-shard step's time depend on which HIP streams the shards got?
(diagnostics): creates a fresh StreamShardedEngine (C3, 65,536 games, two
shards) over and over in one process, as tools/forms_ab.py does per variant,
and times each one's 128-tick step; then re-times the first engine's step.
Prints one JSON line per engine with the shard streams' handles.

    python tools/stream_pairs.py > stream_pairs.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def time_step(torch, e, go, reps=8):
    e.fork()
    for _ in range(2):
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
    return s.elapsed_time(f) * 1e3 / reps


def main():
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import StreamShardedEngine
    dev = torch.device("cuda", 0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    keep = None
    for k in range(n):
        e = StreamShardedEngine(EnvConfig.c3(), 65536, seed=5, device=dev, n_streams=2)
        o, a = e.trajectory_buffers(128)
        go = e.rollout_launcher(128, 1, 1, obs=o, act=a)
        us = time_step(torch, e, go)
        print(json.dumps({"engine": k, "streams": [hex(s.cuda_stream) for s in e.streams],
                          "stream_ids": [int(s.stream_id) for s in e.streams],
                          "us_per_step": round(us, 2)}), flush=True)
        if keep is None:
            keep = (e, o, a, go)
        else:
            del e, o, a, go
    e, o, a, go = keep
    print(json.dumps({"engine": 0, "again": True, "us_per_step": round(time_step(torch, e, go), 2)}),
          flush=True)


if __name__ == "__main__":
    main()
