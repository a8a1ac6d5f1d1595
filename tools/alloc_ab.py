"""VecEnv.step's fresh-output path (diagnostics, round 5): four torch.empty
calls per step against one byte buffer carved into the four outputs by views,
timed as bench.py's vecenv_step extra (C3, 65,536 games, 400 eager steps,
wall clock), both around the same pre-bound orx_env_step_ex launcher.

    python tools/alloc_ab.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from optimax_rogue_amd import EnvConfig, VecEnv
    dev = torch.device("cuda", 0)
    B = 65536
    env = VecEnv(EnvConfig.c3(), B, seed=3, device=dev, opponent=1)
    pool = torch.randint(1, 6, (16, B), dtype=torch.int64, device=dev)
    env.step(pool[0])
    launch = env._launch
    nbytes = B * (56 + 4 + 4 + 1)

    def four(a):
        obs = torch.empty((B, 14), dtype=torch.int32, device=dev)
        rew = torch.empty(B, dtype=torch.float32, device=dev)
        done = torch.empty(B, dtype=torch.bool, device=dev)
        st = torch.empty(B, dtype=torch.int32, device=dev)
        launch(a.data_ptr(), 8, 1, obs.data_ptr(), rew.data_ptr(), done.data_ptr(), st.data_ptr(),
               None)
        return obs, rew, done, st

    def one(a):
        buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        obs = buf[:B * 56].view(torch.int32).view(B, 14)
        rew = buf[B * 56:B * 60].view(torch.float32)
        st = buf[B * 60:B * 64].view(torch.int32)
        done = buf[B * 64:].view(torch.bool)
        launch(a.data_ptr(), 8, 1, obs.data_ptr(), rew.data_ptr(), done.data_ptr(), st.data_ptr(),
               None)
        return obs, rew, done, st

    for rnd in range(3):
        for name, fn in (("four_allocs", four), ("one_alloc_views", one)):
            for k in range(20):
                fn(pool[k % 16])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(400):
                fn(pool[k % 16])
            torch.cuda.synchronize()
            print(json.dumps({"round": rnd, "form": name,
                              "us_per_step": round((time.perf_counter() - t0) / 400 * 1e6, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
