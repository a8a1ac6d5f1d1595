"""Launch sequence for rocprofv3 counter passes (profiles/README.md):
  rollout at the bench config (C3, B=65536, 128 ticks with obs/act, x4:
  rollout_kernel<8, true, false>), then policy_kernel + step_kernel<8> at B=2^21
  (x6) and the plain rollout_kernel<8, true> at 2^21 x 20 ticks (x2)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from optimax_rogue_amd import EnvConfig
from optimax_rogue_amd.engine import BatchedEngine

dev = torch.device("cuda", 0)
B, T = 65536, 128
e = BatchedEngine(EnvConfig.c3(), B, seed=3, device=dev)
obs = torch.empty((T, 14, B), dtype=torch.int32, device=dev)
act = torch.empty((T, B, 2), dtype=torch.int8, device=dev)
e.rollout(T, 1, 1, obs=obs, act=act)
for _ in range(3):
    e.rollout(T, 1, 1, obs=obs, act=act)
torch.cuda.synchronize()
del e, obs, act
BL = 1 << 21
e = BatchedEngine(EnvConfig.c3(), BL, seed=3, device=dev)
for _ in range(6):
    e.step(e.policy(1, 1))
T = 20
obs = torch.empty((T, 14, BL), dtype=torch.int32, device=dev)
act = torch.empty((T, BL, 2), dtype=torch.int8, device=dev)
for _ in range(2):
    e.rollout(T, 1, 1, obs=obs, act=act)
torch.cuda.synchronize()
print("done")
