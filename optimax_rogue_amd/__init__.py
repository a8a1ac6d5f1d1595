"""optimax_rogue_amd -- MI355X-native batched step engine for the Optimax Rogue
per-tick updater (reference: optimax_rogue/logic + optimax_rogue/game).

Host side is Python; the tick, reset and bot policies are HIP kernels for
gfx950 in liborx.so, reached through the C-ABI declared in include/orx.h.
"""
from .config import EnvConfig
from .dungeons import DungeonBank
from .enums import (CombatFlag, DungeonDespawningStrategy, Move, NpcPolicy, OBS_FIELDS, Policy,
                    StartMode, Tile, UpdateResult)

__all__ = ["EnvConfig", "DungeonBank", "Move", "UpdateResult", "DungeonDespawningStrategy", "Tile", "CombatFlag",
           "StartMode", "Policy", "NpcPolicy", "OBS_FIELDS", "BatchedEngine", "StreamShardedEngine", "BatchedUpdater",
           "VecEnv"]


def __getattr__(name):
    # lazy: importing the package must not require torch / the built library
    if name in ("BatchedEngine", "StreamShardedEngine"):
        from . import engine
        return getattr(engine, name)
    if name == "BatchedUpdater":
        from .updater import BatchedUpdater
        return BatchedUpdater
    if name == "VecEnv":
        from .vecenv import VecEnv
        return VecEnv
    raise AttributeError(name)
