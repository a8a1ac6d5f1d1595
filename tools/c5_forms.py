"""C5 on one GPU (131,072 games, 128x128, 2x StaircaseBot) in several launch
forms, and the learner's orx_env_step at 2^21 games (diagnostics, round 5).

Forms: one launch (the plan's one-lane form at 64 games per wave), 2 and 4
stream shards with the plan's choice, and 2 / 4 stream shards forced paired at
32 / 16 games per wave (ORX_ROLLOUT_LANES, read per launch).  Each timed as the
headline step: one fork, 3 warmups, 20 back-to-back 128-tick steps, one join,
HIP events around them.

    python tools/c5_forms.py > c5_forms.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def step_us(torch, e, go, reps=20):
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
    return s.elapsed_time(f) * 1e3 / reps


def main():
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine, StreamShardedEngine
    from optimax_rogue_amd.enums import EXT_SEPARATION_DAMAGE, OBS_FIELDS
    dev = torch.device("cuda", 0)
    T = 128
    which = os.environ.get("C5_FORMS", "c5,env").split(",")
    if "c5" in which:
        forms = [(1, None), (2, None), (2, "32"), (4, None), (4, "16"), (4, "32")]
        for rnd in range(2):
            for sep in (0, 1):
                cfg = EnvConfig.c5()
                if sep:
                    cfg.flags, cfg.sep_period = EXT_SEPARATION_DAMAGE, 8
                for streams, lanes in forms:
                    if lanes:
                        os.environ["ORX_ROLLOUT_LANES"] = lanes
                    else:
                        os.environ.pop("ORX_ROLLOUT_LANES", None)
                    e = StreamShardedEngine(cfg, 131072, seed=5, device=dev, n_streams=streams)
                    o, a = e.trajectory_buffers(T)
                    go = e.rollout_launcher(T, 2, 2, obs=o, act=a)
                    us = step_us(torch, e, go)
                    print(json.dumps({"round": rnd, "sep": sep, "streams": streams,
                                      "lanes_env": lanes, "shape": e.rollout_shape(2, 2),
                                      "us_per_step": round(us, 2),
                                      "bytes_per_step": 131072 * (T * 58 + 144),
                                      "frac": 131072 * (T * 58 + 144) / us / 8e6}), flush=True)
                    del e, o, a, go
                    torch.cuda.empty_cache()
        os.environ.pop("ORX_ROLLOUT_LANES", None)
    if "env" in which:
      for direct in ("0", "1", "0"):   # rows through LDS (the default) / direct stores
        os.environ["ORX_ENV_DIRECT_ROWS"] = direct
        for B in (65536, 1 << 21):
            cfg = EnvConfig.c3()
            eng = BatchedEngine(cfg, B, seed=3, device=dev)
            acts = torch.randint(1, 6, (B,), dtype=torch.int64, device=dev)
            obs = torch.empty((B, len(OBS_FIELDS)), dtype=torch.int32, device=dev)
            rew = torch.empty(B, dtype=torch.float32, device=dev)
            done = torch.empty(B, dtype=torch.bool, device=dev)
            stat = torch.empty(B, dtype=torch.int32, device=dev)
            for _ in range(5):
                eng.env_step(acts, 1, obs, rew, done, stat)
            evs = []
            for _ in range(30):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                eng.env_step(acts, 1, obs, rew, done, stat)
                b.record()
                evs.append((a, b))
            torch.cuda.synchronize()
            d = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
            print(json.dumps({"env_step_games": B, "direct_rows": direct,
                              "us_median": round(d[len(d) // 2], 2),
                              "us_min": round(d[0], 2)}), flush=True)
            del eng, acts, obs, rew, done, stat
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
