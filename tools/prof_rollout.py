"""Runs fused-rollout launches for counter collection.

usage: prof_rollout.py [B] [policy] [npcs] [obs: 1|0]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from optimax_rogue_amd import EnvConfig, _lib

if os.environ.get("ORX_LIB_OVERRIDE"):  # diagnostics: profile another liborx build
    _lib.LIB_PATH = os.path.abspath(os.environ["ORX_LIB_OVERRIDE"])
from optimax_rogue_amd.engine import BatchedEngine

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
pol = int(sys.argv[2]) if len(sys.argv) > 2 else 1
K = int(sys.argv[3]) if len(sys.argv) > 3 else 8
with_obs = (sys.argv[4] != "0") if len(sys.argv) > 4 else True
dev = torch.device("cuda", 0)
e = BatchedEngine(EnvConfig(width=64, height=64, n_npcs=K), B, seed=3, device=dev)
T = int(os.environ.get("ORX_PROF_TICKS", "50"))
obs = torch.empty((T, 14, B), dtype=torch.int32, device=dev) if with_obs else None
act = torch.empty((T, B, 2), dtype=torch.int8, device=dev) if with_obs else None
for _ in range(3):
    e.rollout(T, pol, pol, obs=obs, act=act)
torch.cuda.synchronize()
print("done")
