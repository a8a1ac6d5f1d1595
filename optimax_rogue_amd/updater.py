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
                 has), or a ``(width, height)`` tuple; or an explicit-grid
                 generator, ``optimax_rogue_amd.dungeons.DungeonBank(layouts)``
                 (the plugin API of worldgen.py:9-26 as a layout bank).
  despawn_strat  DungeonDespawningStrategy (updater.py:47-50); ValueError for
                 anything else (updater.py:257).
  max_ticks      None / 0 = no limit (updater.py:158).
  game_start     "together" (TogetherGameStartGenerator) or
                 ("separated", p1_depth, p2_depth) (SeparatedGameStartGenerator).
  npc_policy     the enemy AI: what a subclass overriding
                 Updater.decide_npc_move (updater.py:165-178) would return --
                 NpcPolicy.Stay (the reference's own hook), Random or Chase
                 (include/orx.h ORX_NPC_*); the engine then resolves the NPCs'
                 moves as the reference's update does (:116-145).
"""
from __future__ import annotations

from typing import Optional

import torch

from .config import EnvConfig
from .engine import BatchedEngine
from .enums import DungeonDespawningStrategy, Move, NpcPolicy, Policy, StartMode


def _dims(dgen):
    """(width, height, layouts or None) of a generator argument."""
    from .dungeons import DungeonBank
    if isinstance(dgen, tuple):
        return int(dgen[0]), int(dgen[1]), None
    if isinstance(dgen, DungeonBank):
        return dgen.width, dgen.height, dgen.layouts
    name = type(dgen).__name__
    if name not in ("EmptyDungeonGenerator",):
        raise ValueError(f"unsupported DungeonGenerator {name}: the engine implements "
                         "EmptyDungeonGenerator (worldgen.py:29-43) and DungeonBank layouts")
    return int(dgen.width), int(dgen.height), None


class BatchedUpdater:
    def __init__(self, dgen, despawn_strat: DungeonDespawningStrategy,
                 max_ticks: Optional[int] = None, *, n_games: int, seed: int = 0,
                 game_offset: int = 0, game_start="together", n_npcs: int = 0,
                 device: Optional[torch.device] = None, autoreset: bool = False,
                 npc_policy: NpcPolicy = NpcPolicy.Stay):
        if int(despawn_strat) not in (1, 2):
            raise ValueError(f"Unknown despawn strat {despawn_strat}")
        w, h, layouts = _dims(dgen)
        cfg = EnvConfig(width=w, height=h, despawn=int(despawn_strat), max_ticks=max_ticks or 0,
                        n_npcs=n_npcs, autoreset=int(autoreset), layouts=layouts,
                        npc_policy=int(NpcPolicy(int(npc_policy))))
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
        return game_state(self.engine.snapshot(), i, self.engine.cfg, bank=self.engine.bank)


class GameUpdater:
    """Per-game ``Updater`` front end: ``update(game_state, m1, m2) ->
    (UpdateResult, [GameStateUpdate])`` with the reference's contract
    (updater.py:76-162): it mutates ``game_state`` in place and returns the
    update list a server broadcasts.  Backed by a one-game BatchedEngine
    (global game id ``game_id``); ``game_state`` must be the object returned by
    ``setup_game()`` (a compat.GameStateView, replicated by applying the
    updates exactly as a client would).  One kernel launch per call: the
    compatibility path, not the throughput path."""

    def __init__(self, dgen, despawn_strat: DungeonDespawningStrategy,
                 max_ticks: Optional[int] = None, *, seed: int = 0, game_id: int = 0,
                 game_start="together", n_npcs: int = 0, device: Optional[torch.device] = None,
                 npc_policy: NpcPolicy = NpcPolicy.Stay):
        self._b = BatchedUpdater(dgen, despawn_strat, max_ticks, n_games=1, seed=seed,
                                 game_offset=game_id, game_start=game_start, n_npcs=n_npcs,
                                 device=device, autoreset=False, npc_policy=npc_policy)
        self.engine = self._b.engine
        self.current_update_order = 0
        self.max_ticks = max_ticks
        self.despawn_strat = self._b.despawn_strat

    def setup_game(self):
        """GameStartGenerator.setup_game: the engine's game as a full GameState view."""
        self.engine.reset()
        return self.engine.game_states([0])[0]

    def update(self, game_state, player1_move, player2_move):
        from .compat import DungeonView
        from .updates import from_events
        eng = self.engine
        Move(int(player1_move)), Move(int(player2_move))  # ValueError like Move(...) would
        pre = {e.iden: e.depth for e in game_state.entities}
        eng.actions[0, 0] = int(player1_move)
        eng.actions[0, 1] = int(player2_move)
        status, ev, n = eng.step(events=True)
        rows = [tuple(int(v) for v in r) for r in ev[0, : int(n[0])].cpu().numpy()]
        snap = eng.snapshot()
        cfg = eng.cfg

        def dungeon_for(depth):
            for p in range(2):
                if int(snap["p_depth"][p][0]) == depth:
                    tiles = (eng.bank.tiles(int(snap["p_layout"][p][0]))
                             if eng.bank is not None else None)
                    return DungeonView(cfg.width, cfg.height, int(snap["st_x"][p][0]),
                                       int(snap["st_y"][p][0]), tiles=tiles)
            raise KeyError(depth)

        ups = from_events(rows, self.current_update_order,
                          cfg.player_damage - cfg.player_armor, pre, dungeon_for,
                          npc_og_damage=cfg.npc_damage - cfg.npc_armor)
        self.current_update_order += len(ups)
        for u in ups:
            u.apply(game_state)
        # despawn (updater.py:295-296) and tick (:148) replicate the server side
        from .compat import world_depths
        keep = set(world_depths(cfg, int(snap["p_depth"][0][0]), int(snap["p_depth"][1][0])))
        for d in [d for d in game_state.world.dungeons if d not in keep]:
            game_state.world.del_at_depth(d)
        game_state.tick = int(snap["tick"][0])
        from .enums import UpdateResult
        return UpdateResult(int(status[0].item())), ups


__all__ = ["BatchedUpdater", "GameUpdater", "Move"]
