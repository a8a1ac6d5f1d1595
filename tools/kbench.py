"""Kernel micro-benchmarks (diagnostics).  Run under
``rocprofv3 --kernel-trace`` and summarize with tools/ktrace_summary.py: the
kernel trace gives true device durations (event timing of a single short
launch includes host submission gaps)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from optimax_rogue_amd import EnvConfig
from optimax_rogue_amd.engine import BatchedEngine


def main():
    dev = torch.device("cuda", 0)
    cfgs = [("c3", EnvConfig.c3()), ("k0_64", EnvConfig(width=64, height=64))]
    for cname, cfg in cfgs:
        for B in (65536, 1 << 20):
            print(f"== {cname} B={B}: reset, policy x20, step x20, step(stay) x20, rollout20 x5, "
                  "rollout20-noobs x5, rollout20-stay x5", flush=True)
            e = BatchedEngine(cfg, B, seed=3, device=dev)
            e.rollout(20, 1, 1)
            stay = torch.full((B, 2), 5, dtype=torch.int8, device=dev)
            for _ in range(20):
                e.policy(1, 1)
            for _ in range(20):
                e.step(e.actions)
            for _ in range(20):
                e.step(stay)
            T = 20
            obs = torch.empty((T, 14, B), dtype=torch.int32, device=dev)
            act = torch.empty((T, B, 2), dtype=torch.int8, device=dev)
            for _ in range(5):
                e.rollout(T, 1, 1, obs=obs, act=act)
            for _ in range(5):
                e.rollout(T, 1, 1)
            for _ in range(5):
                e.rollout(T, 3, 3, obs=obs, act=act)
            torch.cuda.synchronize()
            del e


if __name__ == "__main__":
    main()
