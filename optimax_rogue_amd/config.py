"""EnvConfig: the construction arguments of the reference's updater and
generators, mirrored by the POD struct orx_cfg_t (include/orx.h).

Reference counterparts:
  Updater(dgen, despawn_strat, max_ticks)           optimax_rogue/logic/updater.py:65-69
  EmptyDungeonGenerator(width, height)              optimax_rogue/logic/worldgen.py:29-43
  TogetherGameStartGenerator(dgen)                  optimax_rogue/logic/worldgen.py:61-87
  SeparatedGameStartGenerator(dgen, p1_depth, p2_depth)  worldgen.py:90-135
  Entity(iden, depth, x, y, 10, 10, 2, 1, [], {})   worldgen.py:85-86
  an explicit-grid DungeonGenerator plugin          worldgen.py:9-26 (``layouts``,
                                                    optimax_rogue_amd.dungeons.DungeonBank)
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional

import numpy as np

from .enums import DungeonDespawningStrategy, StartMode

CFG_FIELDS = ("width", "height", "despawn", "max_ticks", "start_mode", "p1_depth", "p2_depth",
              "n_npcs", "npc_health", "npc_damage", "npc_armor", "player_health",
              "player_damage", "player_armor", "autoreset", "flags", "n_layouts", "sep_period",
              "rng", "mana_max", "mana_regen", "mana_per_point", "xp_per_kill", "xp_per_level",
              "item_drop_pct", "item_bonus", "item_slots", "combat_cooldown", "npc_policy")


class OrxCfg(ctypes.Structure):
    """ctypes mirror of orx_cfg_t (field order checked against include/orx.h)."""
    _fields_ = [(f, ctypes.c_int32) for f in CFG_FIELDS]


@dataclasses.dataclass
class EnvConfig:
    width: int = 32
    height: int = 32
    despawn: int = DungeonDespawningStrategy.Unreachable
    max_ticks: int = 1000           # 0 / None = never time out
    start_mode: int = StartMode.Together
    p1_depth: int = 0               # Separated start only
    p2_depth: int = 1000            # reference default, worldgen.py:101
    n_npcs: int = 0                 # "enemies": NPCs placed at reset (build-defined spawner)
    npc_health: int = 3
    npc_damage: int = 1
    npc_armor: int = 0
    player_health: int = 10
    player_damage: int = 2
    player_armor: int = 1
    autoreset: int = 1
    flags: int = 0                  # enums.EXT_* build extensions (readme-only mechanics)
    sep_period: int = 0             # EXT_SEPARATION_DAMAGE: ticks per +1 damage
    # word source: RNG_PHILOX (keyed streams, batch/sharding invariant) or
    # RNG_MT19937 (stock seeding: each game's own random / np.random state
    # seeded with seed + game id, consumed in the reference's call order)
    rng: int = 0
    # the readme's character mechanics (flags EXT_MANA / EXT_HEAL /
    # EXT_LEVELING / EXT_ITEMS; readme.md:44, 72, 74).  The readme names no
    # numbers, so every one is a parameter; these defaults are the build's.
    mana_max: int = 9               # manabar; an attack or a heal spends up to a third
    mana_regen: int = 1             # mana regained per tick
    mana_per_point: int = 1         # mana per point of damage / health
    xp_per_kill: int = 1            # experience per NPC kill
    xp_per_level: int = 3           # experience per level (a level refills health, mana)
    item_drop_pct: int = 50         # chance (%) that a dying NPC drops an item
    item_bonus: int = 1             # flat bonus of an item (damage or max health)
    item_slots: int = 3             # items a player can hold
    combat_cooldown: int = 3        # EXT_README_COMBAT: ticks after a mutual attack (readme: 3)
    # the enemy AI (Updater.decide_npc_move, updater.py:165-178): enums.NpcPolicy
    # STAY (the reference's default), RANDOM or CHASE (include/orx.h ORX_NPC_*)
    npc_policy: int = 0
    # explicit-grid dungeon generator: [L, W, H] Tile codes (None =
    # EmptyDungeonGenerator).  spawn_dungeon(depth) returns layout randint(L).
    layouts: Optional[np.ndarray] = dataclasses.field(default=None, repr=False, compare=False)

    @property
    def n_layouts(self) -> int:
        return 0 if self.layouts is None else int(len(self.layouts))

    def to_c(self) -> OrxCfg:
        vals = {f: int(getattr(self, f) or 0) for f in CFG_FIELDS}
        return OrxCfg(**vals)

    def to_dict(self) -> dict:
        return {f: int(getattr(self, f) or 0) for f in CFG_FIELDS}

    @classmethod
    def from_dict(cls, d: dict, layouts=None) -> "EnvConfig":
        """Fields of CFG_FIELDS (n_layouts is derived from ``layouts``)."""
        kw = {k: v for k, v in d.items() if k in CFG_FIELDS and k != "n_layouts"}
        if layouts is None:
            layouts = d.get("layouts")
        return cls(**kw, layouts=None if layouts is None else np.asarray(layouts, np.uint8))

    # --- the BASELINE.json configurations -------------------------------
    @classmethod
    def c1(cls) -> "EnvConfig":
        """Single game, 2x RandomBot, 32x32 (CPU plumbing config)."""
        return cls(width=32, height=32)

    @classmethod
    def c2(cls) -> "EnvConfig":
        """batch=4096, 32x32, random actions."""
        return cls(width=32, height=32)

    @classmethod
    def c3(cls) -> "EnvConfig":
        """batch=65536, 64x64 with enemies (K=8 NPCs; items have no reference semantics)."""
        return cls(width=64, height=64, n_npcs=8)

    @classmethod
    def c4(cls) -> "EnvConfig":
        """batch=524288 over 8 GPUs, C3 settings."""
        return cls.c3()

    @classmethod
    def c5(cls) -> "EnvConfig":
        """128x128 multi-depth with the staircase ("ladder") policy."""
        return cls(width=128, height=128)
