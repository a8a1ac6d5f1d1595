"""A/B of the per-tick step across liborx builds (diagnostics): for every
library path given, a fresh child process times orx_step (the reference's
`Updater.update` drop-in) on C3 at 2^21 and 65,536 games, actions drawn by
orx_policy beforehand (RandomBots), HIP events around `reps` launches.
Libraries alternate, `--reps=N` rounds.

    python tools/ab_step.py old.so new.so [--reps=3]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    sys.path.insert(0, ROOT)
    import torch
    from optimax_rogue_amd import _lib, EnvConfig
    _lib.LIB_PATH = os.path.abspath(lib)
    from optimax_rogue_amd.engine import BatchedEngine
    dev = torch.device("cuda", 0)
    out = {"lib": lib}
    for B, reps in ((1 << 21, 20), (65536, 50)):
        e = BatchedEngine(EnvConfig.c3(), B, seed=1, device=dev)
        e.rollout(20, 1, 1)
        e.policy(1, 1)
        for _ in range(3):
            e.step(e.actions)
        torch.cuda.synchronize()
        s, f = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            e.step(e.actions)
        f.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(f) * 1e3 / reps
        out[f"step_B{B}"] = {"us_per_launch": round(us, 2), "env_steps_per_s": B / us * 1e6}
        # the same launches captured in a HIP graph (no host launch cost)
        g = torch.cuda.CUDAGraph()
        sg = torch.cuda.Stream(device=dev)
        sg.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(sg):
            with torch.cuda.graph(g, stream=sg):
                for _ in range(reps):
                    e.step(e.actions)
        torch.cuda.current_stream().wait_stream(sg)
        g.replay()
        torch.cuda.synchronize()
        s.record()
        g.replay()
        f.record()
        torch.cuda.synchronize()
        out[f"step_B{B}"]["graph_us_per_launch"] = round(s.elapsed_time(f) * 1e3 / reps, 2)
    print(json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    libs = [a for a in sys.argv[1:] if not a.startswith("--")]
    reps = 3
    for a in sys.argv[1:]:
        if a.startswith("--reps="):
            reps = int(a.split("=", 1)[1])
    for _ in range(reps):
        for lib in libs:
            r = subprocess.run([sys.executable, __file__, "--child", lib], capture_output=True,
                               text=True, timeout=300)
            if r.returncode != 0:
                raise SystemExit(f"{lib}: {r.stderr[-2000:]}")
            print(r.stdout.strip().splitlines()[-1], flush=True)


if __name__ == "__main__":
    main()
