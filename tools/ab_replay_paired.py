"""A/B of orx_step_n's forms at the bench's replay shape (C3, 65,536 games,
128-tick uniform move logs, int32 rows): the one-lane replay_kernel
(ORX_REPLAY_PAIRED=0), the paired LOG form as one launch (=1, 32 games per
wave), and the paired form as two 32,768-game stream shards (the headline's
recipe; each shard's log generated for it).  Every form's rows are checked
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
    from optimax_rogue_amd.engine import BatchedEngine
    dev = torch.device("cuda", 0)
    B, T, reps = 65536, 128, 10
    cfg = EnvConfig.c3()
    g = torch.Generator(device="cpu").manual_seed(11)
    log = torch.randint(1, 6, (T, B, 2), generator=g, dtype=torch.int8).to(dev)
    half = B // 2
    logs2 = [log[:, :half].contiguous(), log[:, half:].contiguous()]

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

    def two_shards():
        os.environ["ORX_REPLAY_PAIRED"] = "1"
        os.environ["ORX_ROLLOUT_LANES"] = "32"
        try:
            from optimax_rogue_amd.engine import shard_streams
            streams = shard_streams(dev, 2)
            engs = [BatchedEngine(cfg, half, seed=3, game_offset=k * half, device=dev)
                    for k in range(2)]
            obs = [torch.empty((T, len(OBS_FIELDS), half), dtype=torch.int32, device=dev)
                   for _ in range(2)]

            def step():
                cur = torch.cuda.current_stream(dev)
                for s in streams:
                    s.wait_stream(cur)
                for e, s, l, o in zip(engs, streams, logs2, obs):
                    with torch.cuda.stream(s):
                        e.step_n(l, obs=o)
                for s in streams:
                    cur.wait_stream(s)
            step()
            torch.cuda.synchronize()
            first = torch.cat([o.cpu() for o in obs], dim=2)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                step()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / reps, first
        finally:
            del os.environ["ORX_REPLAY_PAIRED"]
            del os.environ["ORX_ROLLOUT_LANES"]

    for r in range(rounds):
        base_us, base = one_launch("0")
        out = {"round": r, "one_lane_us": base_us}
        us, rows = one_launch("1")
        out["paired_one_launch_us"] = us
        out["paired_one_launch_equal"] = bool(torch.equal(rows, base))
        us, rows = two_shards()
        out["paired_two_shards_us"] = us
        out["paired_two_shards_equal"] = bool(torch.equal(rows, base))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
