"""Host overhead of one engine call (diagnostics): times n back-to-back
orx_rollout launches of 1 tick over 256 games (device work ~negligible) and
the pieces of the Python call path."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from optimax_rogue_amd import EnvConfig
from optimax_rogue_amd.engine import BatchedEngine

dev = torch.device("cuda", 0)
e = BatchedEngine(EnvConfig.c3(), 256, seed=1, device=dev)
obs = torch.empty((1, 14, 256), dtype=torch.int32, device=dev)
act = torch.empty((1, 256, 2), dtype=torch.int8, device=dev)
n = 2000
for _ in range(100):
    e.rollout(1, 1, 1, obs=obs, act=act)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    e.rollout(1, 1, 1, obs=obs, act=act)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"rollout call: {(t1 - t0) / n * 1e6:.1f} us/call enqueue, {(t2 - t0) / n * 1e6:.1f} us/call total")
t0 = time.perf_counter()
for _ in range(n):
    with torch.cuda.device(dev):
        pass
t1 = time.perf_counter()
print(f"torch.cuda.device ctx: {(t1 - t0) / n * 1e6:.2f} us")
t0 = time.perf_counter()
for _ in range(n):
    torch.cuda.current_stream(dev).cuda_stream
t1 = time.perf_counter()
print(f"current_stream: {(t1 - t0) / n * 1e6:.2f} us")
t0 = time.perf_counter()
for _ in range(n):
    a = torch.cuda.Event(enable_timing=True)
    a.record()
t1 = time.perf_counter()
print(f"Event()+record: {(t1 - t0) / n * 1e6:.2f} us")
