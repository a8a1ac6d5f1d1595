"""A/B of orx_step_n's forms at the bench's replay shape (C3, 65,536 games,
128-tick uniform move logs, int32 rows): the one-lane replay_kernel
(ORX_REPLAY_PAIRED=0), the paired LOG form as one launch (=1, 32 games per
wave), and orx_step_n as two 32,768-game stream shards
(StreamShardedEngine.replay_launcher, the headline's recipe: launches back to
back per shard, one fork / join around the timed ones; the plan's lanes and
32 forced).  Every form's rows are checked
equal to the one-lane form's.  Prints one JSON line per form and round.

    python tools/ab_replay_paired.py [rounds]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    import torch
    from optimax_rogue_amd import EnvConfig, OBS_FIELDS
    from optimax_rogue_amd.engine import BatchedEngine, StreamShardedEngine, shard_streams
    dev = torch.device("cuda", 0)
    shard_streams(dev, 2)   # first, as bench.py's headline engine gets them
    B, T, reps = 65536, 128, 10
    cfg = EnvConfig.c3()
    g = torch.Generator(device="cpu").manual_seed(11)
    log = torch.randint(1, 6, (T, B, 2), generator=g, dtype=torch.int8).to(dev)

    def one_launch(env):
        os.environ["ORX_REPLAY_PAIRED"] = env
        try:
            eng = BatchedEngine(cfg, B, seed=3, device=dev)
            obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
            eng.step_n(log, obs=obs)
            torch.cuda.synchronize()
            first = obs.cpu()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                eng.step_n(log, obs=obs)
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / reps, first
        finally:
            del os.environ["ORX_REPLAY_PAIRED"]

    def two_shards(lanes):
        # the headline's recipe: the process's shard streams (created first,
        # in main), each shard's launches back to back on its stream, one fork
        # before and one join after the timed launches
        if lanes:
            os.environ["ORX_ROLLOUT_LANES"] = lanes
        try:
            se = StreamShardedEngine(cfg, B, seed=3, device=dev, n_streams=2)
            logs = se.split_log(log)
            obs, _ = se.trajectory_buffers(T)
            go = se.replay_launcher(logs, obs)
            se.fork()
            go()
            se.join()
            torch.cuda.synchronize()
            first = torch.cat([o.cpu() for o in obs], dim=2)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            se.fork()
            for _ in range(reps):
                go()
            se.join()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / reps, first
        finally:
            if lanes:
                del os.environ["ORX_ROLLOUT_LANES"]

    for r in range(rounds):
        base_us, base = one_launch("0")
        out = {"round": r, "one_lane_us": base_us}
        us, rows = one_launch("1")
        out["paired_one_launch_us"] = us
        out["paired_one_launch_equal"] = bool(torch.equal(rows, base))
        for lanes in ("", "32"):
            us, rows = two_shards(lanes)
            key = "two_shards" + ("_lanes" + lanes if lanes else "")
            out[key + "_us"] = us
            out[key + "_equal"] = bool(torch.equal(rows, base))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
