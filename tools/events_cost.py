"""What the update-event list costs (diagnostics): orx_step against
orx_step_events at C3 (65,536 and 2^21 games, RandomBot actions drawn by
orx_policy beforehand, one pair reused), median of 30 launches between HIP
events each, and the events' own bytes per game-tick (8 records x 16 B + the
count, written whether or not a record is used).

    python tools/events_cost.py [lib.so]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import timed_launches
    from optimax_rogue_amd import _lib, EnvConfig
    if len(sys.argv) > 1:
        _lib.LIB_PATH = os.path.abspath(sys.argv[1])
    from optimax_rogue_amd.engine import BatchedEngine
    dev = torch.device("cuda", 0)
    out = {"lib": _lib.LIB_PATH}
    for B in (65536, 1 << 21):
        eng = BatchedEngine(EnvConfig.c3(), B, seed=3, device=dev)
        a = eng.policy(1, 1).clone()
        eng.step(a)
        eng.step(a, events=True)
        s = sorted(timed_launches(torch, lambda: eng.step(a), 30))
        e = sorted(timed_launches(torch, lambda: eng.step(a, events=True), 30))
        out[str(B)] = {"step_us": round(s[15] * 1e6, 2), "step_events_us": round(e[15] * 1e6, 2),
                       "max_events": eng.max_events()}
        del eng, a
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
