"""Diagnostics: the bench step (two stream shards x one 128-tick rollout
launch) timed as plain launches, as one HIP graph per step, and as one
graph holding all K steps (HIP events on the current stream).

    python tools/graph_step.py [steps]
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
    launch = eng.rollout_launcher(128, 1, 1, obs=obs, act=act)

    def timed(fn, reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        fn(reps)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / reps

    def plain(n):
        eng.fork()
        for _ in range(n):
            launch()
        eng.join()

    for _ in range(2):
        plain(5)
    res = {"plain_us_per_step": timed(plain, K)}
    # one graph per step: fork, both shards' launches, join
    g1 = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        eng2 = eng  # the launcher bound the shard streams at creation
        with torch.cuda.graph(g1, stream=s):
            eng2.fork()
            launch()
            eng2.join()
    torch.cuda.current_stream().wait_stream(s)
    g1.replay()

    def per_step(n):
        for _ in range(n):
            g1.replay()
    res["graph_per_step_us"] = timed(per_step, K)
    gK = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(gK, stream=s):
            eng.fork()
            for _ in range(K):
                launch()
            eng.join()
    torch.cuda.current_stream().wait_stream(s)
    gK.replay()
    res["graph_all_steps_us_per_step"] = timed(lambda n: [gK.replay() for _ in range(n)], 3) / K
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
