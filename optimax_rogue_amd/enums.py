"""Integer enums of the reference, same names and values.

Move                       optimax_rogue/logic/moves.py:6-12
UpdateResult               optimax_rogue/logic/updater.py:16-21
DungeonDespawningStrategy  optimax_rogue/logic/updater.py:47-50
Tile                       optimax_rogue/game/world.py:10-17
CombatFlag                 optimax_rogue/game/modifiers.py:7-12
"""
import enum


class Move(enum.IntEnum):
    Up = 1
    Right = 2
    Down = 3
    Left = 4
    Stay = 5


class UpdateResult(enum.IntEnum):
    InProgress = 1
    Player1Win = 2
    Player2Win = 3
    Tie = 4


class DungeonDespawningStrategy(enum.IntEnum):
    Unreachable = 1
    Unused = 2


class Tile(enum.IntEnum):
    Ground = 1
    Wall = 2
    StaircaseDown = 3


class CombatFlag(enum.IntEnum):
    Block = 1
    Ambush = 2
    Flee = 3
    Parry = 4


class StartMode(enum.IntEnum):
    """Which GameStartGenerator plugin (optimax_rogue/logic/worldgen.py:61-135)."""
    Together = 1
    Separated = 2


class Policy(enum.IntEnum):
    """On-device action producers (optimax_rogue_bots/randombot.py, staircasebot.py)."""
    NONE = 0
    Random = 1
    Staircase = 2
    Stay = 3


class NpcPolicy(enum.IntEnum):
    """The enemy AI, EnvConfig.npc_policy (include/orx.h ORX_NPC_*): the
    reference's hook Updater.decide_npc_move (updater.py:165-178) returns Stay;
    RANDOM and CHASE are the AIs tests/golden/make_golden.NpcAiUpdater plugs
    into it (the reference then resolves the moves)."""
    Stay = 0
    Random = 1
    Chase = 2


# build-only per-game status codes (include/orx.h)
STATUS_BAD_ACTION = 16
STATUS_RNG_EXHAUSTED = 17

# build extensions (orx_cfg_t.flags, include/orx.h ORX_EXT_*): readme-only
# mechanics, off by default, parity unpinned
EXT_SEPARATION_DAMAGE = 1
EXT_RANDOM_DOUBLE_DEATH = 2
# the readme's character mechanics (readme.md:44, 72, 74), parameters in EnvConfig
EXT_MANA = 4          # up to 1/3 of the manabar converted into attack damage
EXT_HEAL = 8          # MOVE_HEAL: a Stay converting up to 1/3 of the manabar into health
EXT_LEVELING = 16     # experience per NPC kill; a level refills health and mana
EXT_ITEMS = 32        # NPC drops with flat bonuses, picked up into finite item spots
EXT_RPG = EXT_MANA | EXT_HEAL | EXT_LEVELING | EXT_ITEMS
EXT_README_COMBAT = 64  # the readme's combat table (half damage, cooldowns, negation)
EXT_CHARACTER = EXT_RPG | EXT_README_COMBAT   # the flags that keep p_rpg
MOVE_HEAL = 6         # action code of a heal (EXT_HEAL only; not a reference Move)
# rows of the p_rpg player-attribute tensor (include/orx.h ORX_RPG_*)
RPG_FIELDS = ("mana", "xp", "damage", "max_health", "items", "cooldown")

# EnvConfig.rng (orx_cfg_t.rng, include/orx.h ORX_RNG_*)
RNG_PHILOX = 0
RNG_MT19937 = 1
# stock-seed mode: depths per player's dstore ring (orx_dstore_depths)
DSTORE_MIN, DSTORE_UNBOUNDED, DSTORE_MAX = 256, 4096, 65536

# per-game event counter rows (include/orx.h ORX_CNT_*)
CNT_COMBAT, CNT_DESCEND, CNT_DUNGEON, CNT_NPC_DEATH = range(4)
N_COUNTERS = 4
MAX_NPCS = 255       # ORX_MAX_NPCS
MAX_REG_NPCS = 16    # ORX_MAX_REG_NPCS: above, the NPCs live in an HBM occupancy grid


def npc_alive_bits(alive, K: int):
    """bool [K, B] from an npc_alive array ([B] for K <= 32, else
    [ceil(K / 32), B] rows of 32 bits)."""
    import numpy as np
    a = np.asarray(alive).astype(np.uint64)
    if a.ndim == 1:
        a = a[None, :]
    k = np.arange(K)
    return ((a[k // 32] >> (k % 32)[:, None].astype(np.uint64)) & 1).astype(bool)

OBS_FIELDS = ("p1_x", "p1_y", "p1_depth", "p1_health", "p2_x", "p2_y", "p2_depth",
              "p2_health", "tick", "status", "p1_stair_x", "p1_stair_y", "p2_stair_x",
              "p2_stair_y")

# trajectory row formats of orx_rollout_ex (include/orx.h ORX_OBS_*): the
# int32 rows above, or the compact uint32 rows (cells as u8 pairs, int16
# healths, tick | status << 27): 24 bytes per env-step instead of 56
OBS_INT32, OBS_COMPACT = 0, 1
OBS_COMPACT_FIELDS = ("cells", "stairs", "health", "p1_depth", "p2_depth", "tick_status")
COMPACT_MAX_STAT = 8000
SEP_PERIOD_MAX = 1 << 24   # ORX_SEP_PERIOD_MAX: cfg.sep_period's upper bound

# update-event records of orx_step_events (include/orx.h ORX_EV_*)
EV_COMBAT, EV_DEATH, EV_POSITION, EV_DUNGEON, EV_HEALTH = 1, 2, 3, 4, 5
MAX_EVENTS = 8
