"""Would a paired (two lanes per game) learner tick pay?  Device time per
launch at 65,536 games (C3), 50 launches captured in one HIP graph, of:

  env_step       orx_env_step_ex with both players' int64 actions ([B][2],
                 no policy), obs rows [B][14], reward, done, status, the
                 refused-action count -- the learner's tick as it is
                 (step_game's literal one-lane tick)
  paired_tick    orx_step_n over a 1-tick log with int32 rows: the paired LOG
                 form (pair_rollout_kernel PM 6, two lanes per game, 32 games
                 per wave) -- the rollout's paired tick on given actions,
                 field-major rows, no reward / done / status outputs
  one_lane_tick  the same through the one-lane replay_kernel
                 (ORX_REPLAY_PAIRED=0)
  step           orx_step alone (state in, state out, no rows)

Prints one JSON line per round.

    python tools/ab_env_paired.py [rounds]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def graph_us(torch, dev, fn, n=50, reps=4):
    fn()
    g = torch.cuda.CUDAGraph()
    sg = torch.cuda.Stream(device=dev)
    sg.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(sg):
        with torch.cuda.graph(g, stream=sg):
            for _ in range(n):
                fn()
    torch.cuda.current_stream().wait_stream(sg)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1e3 / (n * reps), 2)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    import torch
    from optimax_rogue_amd import EnvConfig, OBS_FIELDS
    from optimax_rogue_amd.engine import BatchedEngine
    dev = torch.device("cuda", 0)
    B = 65536
    cfg = EnvConfig.c3()
    for r in range(rounds):
        out = {"round": r, "games": B}
        eng = BatchedEngine(cfg, B, seed=3, device=dev)
        la = torch.randint(1, 6, (B, 2), dtype=torch.int64, device=dev)
        lo = torch.empty((B, len(OBS_FIELDS)), dtype=torch.int32, device=dev)
        lr = torch.empty(B, dtype=torch.float32, device=dev)
        ld = torch.empty(B, dtype=torch.bool, device=dev)
        ls = torch.empty(B, dtype=torch.int32, device=dev)
        lb = torch.zeros(1, dtype=torch.int32, device=dev)
        out["env_step_us"] = graph_us(torch, dev, lambda: eng.env_step(la, 0, lo, lr, ld, ls, lb))
        log = la.to(torch.int8).reshape(1, B, 2).contiguous()
        rows = torch.empty((1, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
        out["paired_tick_us"] = graph_us(torch, dev, lambda: eng.step_n(log, obs=rows))
        os.environ["ORX_REPLAY_PAIRED"] = "0"
        try:
            out["one_lane_tick_us"] = graph_us(torch, dev, lambda: eng.step_n(log, obs=rows))
        finally:
            del os.environ["ORX_REPLAY_PAIRED"]
        a8 = log[0]
        out["step_us"] = graph_us(torch, dev, lambda: eng.step(a8))
        print(json.dumps(out), flush=True)
        del eng


if __name__ == "__main__":
    main()
