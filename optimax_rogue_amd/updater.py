"""BatchedUpdater: the reference Updater's interface over a batch of games.

Reference: ``Updater(dgen, despawn_strat, max_ticks)`` and
``Updater.update(game_state, player1_move, player2_move) -> (UpdateResult, updates)``
(optimax_rogue/logic/updater.py:52-162).  Batched form: the engine owns every
game's state (the reference mutates ``game_state`` in place, so holding it is
the same contract), and ``update(player1_moves, player2_moves)`` advances all
games one tick and returns their UpdateResult codes.

Construction mirrors the reference's plugins:
  dgen           EmptyDungeonGenerator(width, height) (worldgen.py:29-43): any
                 object with ``width``/``height`` whose class is named
                 ``EmptyDungeonGenerator`` (the only generator the reference
                 has), or a ``(width, height)`` tuple.
  despawn_strat  DungeonDespawningStrategy (updater.py:47-50); ValueError for
                 anything else (updater.py:257).
  max_ticks      None / 0 = no limit (updater.py:158).
  game_start     "together" (TogetherGameStartGenerator) or
                 ("separated", p1_depth, p2_depth) (SeparatedGameStartGenerator).
"""
from __future__ import annotations

from typing import Optional

import torch

from .config import EnvConfig
from .engine import BatchedEngine
from .enums import DungeonDespawningStrategy, Move, Policy, StartMode


def _dims(dgen):
    if isinstance(dgen, tuple):
        return int(dgen[0]), int(dgen[1])
    name = type(dgen).__name__
    if name not in ("EmptyDungeonGenerator",):
        raise ValueError(f"unsupported DungeonGenerator {name}: the engine implements "
                         "EmptyDungeonGenerator (worldgen.py:29-43)")
    return int(dgen.width), int(dgen.height)


class BatchedUpdater:
    def __init__(self, dgen, despawn_strat: DungeonDespawningStrategy,
                 max_ticks: Optional[int] = None, *, n_games: int, seed: int = 0,
                 game_offset: int = 0, game_start="together", n_npcs: int = 0,
                 device: Optional[torch.device] = None, autoreset: bool = False):
        if int(despawn_strat) not in (1, 2):
            raise ValueError(f"Unknown despawn strat {despawn_strat}")
        w, h = _dims(dgen)
        cfg = EnvConfig(width=w, height=h, despawn=int(despawn_strat), max_ticks=max_ticks or 0,
                        n_npcs=n_npcs, autoreset=int(autoreset))
        if game_start != "together":
            kind, d1, d2 = game_start
            if kind != "separated":
                raise ValueError(f"unknown game start {game_start}")
            cfg.start_mode, cfg.p1_depth, cfg.p2_depth = StartMode.Separated, int(d1), int(d2)
        self.engine = BatchedEngine(cfg, n_games, seed=seed, game_offset=game_offset,
                                    device=device)
        self.max_ticks = max_ticks
        self.despawn_strat = DungeonDespawningStrategy(int(despawn_strat))

    @property
    def n_games(self) -> int:
        return self.engine.B

    def update(self, player1_moves, player2_moves) -> torch.Tensor:
        """One tick of every game (Updater.update).  Moves: Move values 1..5,
        one per game (sequence, numpy array or tensor).  Returns the int32
        UpdateResult tensor (device; ORX status >= 16 for invalid moves)."""
        dev = self.engine.device
        m1 = torch.as_tensor(player1_moves, dtype=torch.int8).to(dev)
        m2 = torch.as_tensor(player2_moves, dtype=torch.int8).to(dev)
        if m1.numel() != self.n_games or m2.numel() != self.n_games:
            raise ValueError("one move per game and player")
        self.engine.actions[:, 0] = m1.reshape(-1)
        self.engine.actions[:, 1] = m2.reshape(-1)
        return self.engine.step()

    def bot_moves(self, p1: Policy = Policy.Random, p2: Policy = Policy.Random) -> torch.Tensor:
        """RandomBot / StaircaseBot moves for every game, on the device."""
        return self.engine.policy(p1, p2)

    def game_state(self, i: int):
        """Game i in the reference GameState schema (compat.GameStateView)."""
        from .compat import game_state
        return game_state(self.engine.snapshot(), i, self.engine.cfg)


__all__ = ["BatchedUpdater", "Move"]
