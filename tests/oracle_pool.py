"""TEST INFRASTRUCTURE: the C oracle over a whole batch, in threads.

A batch of B games (global ids offset .. offset + B - 1) as N contiguous
chunks, each its own oracle (oracle/orx_oracle.c through the ctypes wrapper;
ctypes releases the GIL inside the C calls, so the chunks advance in
parallel).  Used to check the engine's timed shapes game by game instead of
by samples (C3: 65,536 games x 1,152 ticks is ~1 s of oracle work on 16
host threads).
"""
from __future__ import annotations

import os
import threading

import numpy as np


def host_threads(cap: int = 16) -> int:
    """Threads for the pool: this process's CPU affinity, at most ``cap``
    (the GPU box's share per GPU)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(cap, n))


class OraclePool:
    def __init__(self, oracle_lib, cfg: dict, n_games: int, seed: int, offset: int = 0,
                 threads: int = 0, layouts=None, episode: int = 0):
        n = threads or host_threads()
        n = max(1, min(n, n_games))
        base, extra = divmod(n_games, n)
        self.bounds = []
        start = 0
        for k in range(n):
            cnt = base + (1 if k < extra else 0)
            self.bounds.append((start, start + cnt))
            start += cnt
        self.B = n_games
        self.oras = [oracle_lib.Oracle(cfg, b - a, seed, offset + a, layouts=layouts)
                     for a, b in self.bounds]
        self.K = self.oras[0].K
        self._run(lambda o, a, b, k: o.reset(episode=np.full(b - a, episode, np.int32)))

    def _run(self, fn):
        errs = []

        def work(k):
            try:
                a, b = self.bounds[k]
                fn(self.oras[k], a, b, k)
            except BaseException as e:   # re-raised in the caller
                errs.append(e)

        th = [threading.Thread(target=work, args=(k,)) for k in range(len(self.oras))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]

    def rollout(self, pol1: int, pol2: int, n_ticks: int) -> None:
        """n_ticks x (policy, step) of every game."""
        self._run(lambda o, a, b, k: o.rollout(pol1, pol2, n_ticks))

    def step(self, actions: np.ndarray) -> None:
        """One step with actions [B, 2] int8."""
        self._run(lambda o, a, b, k: o.step(actions[a:b]))

    def policy(self, pol1: int, pol2: int, actions: np.ndarray = None) -> np.ndarray:
        """The bots' moves for every game (policy 0 keeps ``actions``' column)."""
        out = np.full((self.B, 2), 5, np.int8) if actions is None else actions.copy()

        def fn(o, a, b, k):
            out[a:b] = o.policy(pol1, pol2, out[a:b])
        self._run(fn)
        return out

    def export(self) -> dict:
        parts = [None] * len(self.oras)

        def fn(o, a, b, k):
            parts[k] = o.export()
        self._run(fn)
        return {k: np.concatenate([p[k] for p in parts], axis=-1) for k in parts[0]}
