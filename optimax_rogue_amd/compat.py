"""Reference-schema views of batched games, for code written against
optimax_rogue's GameState (bots, spectators, tools).

``game_state(snapshot, i, cfg)`` materializes game ``i`` of an engine snapshot
as an object with the reference's attribute surface:

  GameState  optimax_rogue/game/state.py:14-62   (tick, player_1_iden/2, world,
             entities, pos_lookup, iden_lookup, player_1/2, view_for, view_spec)
  World      optimax_rogue/game/world.py:101-135 (dungeons dict, get_at_depth)
  Dungeon    optimax_rogue/game/world.py:19-66   (tiles[W, H] int32, width,
             height, is_blocked, get_unblocked, staircase)
  Entity     optimax_rogue/game/entities.py:17-74 (iden, depth, x, y, health,
             base stats, max_health/damage/armor attribles with .value)

so that ``Bot.move(game_state)`` implementations (optimax_rogue_bots/bot.py:6-38,
randombot.py, staircasebot.py) run unchanged via ``BotDriver``.

World contents: the dungeons of the players' current depths (the engine keeps
no other dungeon; a bot's view, GameState.view_for, only ever holds its own
depth).  This is the slow, per-game compatibility path; the throughput path
is the on-device policy kernels (Policy.Random / Policy.Staircase).
"""
from __future__ import annotations

import json
import struct
from typing import Dict, List, Optional, Sequence

import numpy as np

from .enums import DungeonDespawningStrategy, Move, StartMode, Tile, UpdateResult

# serializer registry names (serializer.py:91-95: module + '.' + underscore(class))
GAME_STATE_IDEN = "optimax_rogue.game.state.game_state"
ENTITY_IDEN = "optimax_rogue.game.entities.entity"


def ascii85(data: bytes) -> bytes:
    """The reference's a85 flavour (a85encode.py:6-28): zero-pad to a multiple
    of 4 bytes, every 4-byte big-endian group -> 5 base-85 digits + 33, no 'z'
    shortcut, nothing truncated."""
    if len(data) % 4:
        data = data + b"\0" * (4 - len(data) % 4)
    out = bytearray()
    for (v,) in struct.iter_unpack(">I", data):
        digits = []
        for _ in range(5):
            v, r = divmod(v, 85)
            digits.append(33 + r)
        out.extend(reversed(digits))
    return bytes(out)


def _json(obj) -> bytes:
    # JsonSerializer.serialize (serializer.py:46-52): sorted keys, default separators
    return json.dumps(obj, sort_keys=True).encode("ascii")


class _Attrible:
    def __init__(self, value: int):
        self.value = value


class EntityView:
    def __init__(self, iden, depth, x, y, health, base_max_health, base_damage, base_armor):
        self.iden, self.depth, self.x, self.y = int(iden), int(depth), int(x), int(y)
        self.health = int(health)
        self.base_max_health, self.base_damage, self.base_armor = (
            int(base_max_health), int(base_damage), int(base_armor))
        self.max_health = _Attrible(self.base_max_health)
        self.damage = _Attrible(self.base_damage)
        self.armor = _Attrible(self.base_armor)
        self.modifiers: list = []
        self.items: dict = {}

    def on_tick(self, game_state) -> None:  # attribles are constant (no Modifier exists)
        pass

    def to_prims(self) -> dict:
        """Entity.to_prims (entities.py:76-88); no modifiers or items exist."""
        return {"iden": self.iden, "x": self.x, "y": self.y, "depth": self.depth,
                "health": self.health, "base_max_health": self.base_max_health,
                "base_damage": self.base_damage, "base_armor": self.base_armor,
                "modifiers": [], "items": {}}

    def serialize(self) -> bytes:
        """serializer.serialize(entity) (serializer.py:150-156)."""
        return _json({"iden": ENTITY_IDEN, "prims": self.to_prims()})

    def __eq__(self, other):  # Entity.__eq__ (entities.py:97-128)
        return isinstance(other, EntityView) and all(
            getattr(self, f) == getattr(other, f) for f in (
                "iden", "depth", "x", "y", "health", "base_max_health", "base_damage",
                "base_armor"))

    def __repr__(self):
        return f"[Entity @ ({self.x}, {self.y})]"


class DungeonView:
    """A Dungeon (world.py:19-99): the EmptyDungeonGenerator layout
    (worldgen.py:33-43) with its staircase, or the given tiles (a dungeon-bank
    layout)."""

    def __init__(self, width: int, height: int, sx: int, sy: int, tiles=None):
        if tiles is not None:
            self.tiles = np.asarray(tiles, np.int32)
            return
        t = np.full((width, height), Tile.Ground.value, np.int32)
        t[[0, -1], :] = Tile.Wall.value
        t[:, [0, -1]] = Tile.Wall.value
        t[sx, sy] = Tile.StaircaseDown.value
        self.tiles = t

    @property
    def width(self):
        return self.tiles.shape[0]

    @property
    def height(self):
        return self.tiles.shape[1]

    def is_blocked(self, x: int, y: int) -> bool:
        if x < 0 or x >= self.width or y < 0 or y >= self.height:
            return True
        return self.tiles[x, y] == Tile.Wall

    def get_unblocked(self) -> np.ndarray:
        return self.tiles != Tile.Wall

    def staircase(self):
        resx, resy = tuple(np.argwhere(self.tiles == Tile.StaircaseDown)[0])
        return int(resx), int(resy)

    def to_prims(self) -> bytes:
        """Dungeon.to_prims (world.py:73-81): W, H big-endian u32, uint8 tiles x-major."""
        return (struct.pack(">II", self.width, self.height) +
                self.tiles.astype(np.uint8).reshape(-1).tobytes())

    def __eq__(self, other):
        return isinstance(other, DungeonView) and np.array_equal(self.tiles, other.tiles)


class WorldView:
    def __init__(self, dungeons: Dict[int, DungeonView]):
        self.dungeons = dungeons

    def get_at_depth(self, ind: int) -> DungeonView:
        return self.dungeons[ind]

    def set_at_depth(self, ind: int, dung: DungeonView) -> None:
        self.dungeons[ind] = dung

    def del_at_depth(self, ind: int) -> None:
        del self.dungeons[ind]

    def shallow_copy_with_layers(self, *layers) -> "WorldView":
        return WorldView({lyr: self.dungeons[lyr] for lyr in layers})

    def to_prims(self) -> bytes:
        """World.to_prims (world.py:142-151): count, then per dungeon (dict order)
        depth u32, length u64, Dungeon.to_prims."""
        out = [struct.pack(">I", len(self.dungeons))]
        for depth, dung in self.dungeons.items():
            d = dung.to_prims()
            out.append(struct.pack(">IQ", depth, len(d)))
            out.append(d)
        return b"".join(out)

    def __eq__(self, other):  # World.__eq__ (world.py:167-175): dict order ignored
        return (isinstance(other, WorldView) and len(self.dungeons) == len(other.dungeons)
                and all(d in other.dungeons and dg == other.dungeons[d]
                        for d, dg in self.dungeons.items()))


class GameStateView:
    def __init__(self, is_authoritative: bool, tick: int, world: WorldView,
                 entities: List[EntityView], player_1_iden: int = 1, player_2_iden: int = 2):
        self.is_authoritative = is_authoritative
        self.tick = int(tick)
        self.player_1_iden, self.player_2_iden = player_1_iden, player_2_iden
        self.world = world
        self.entities = entities
        self.pos_lookup = {(e.depth, e.x, e.y): e for e in entities}
        self.iden_lookup = {e.iden: e for e in entities}

    @property
    def player_1(self) -> EntityView:
        return self.iden_lookup[self.player_1_iden]

    @property
    def player_2(self) -> EntityView:
        return self.iden_lookup[self.player_2_iden]

    def on_tick(self) -> None:
        pass

    # GameState mutators (state.py:64-88), used by update.apply()
    def move_entity(self, entity, newdepth, newx, newy):
        del self.pos_lookup[(entity.depth, entity.x, entity.y)]
        entity.depth, entity.x, entity.y = int(newdepth), int(newx), int(newy)
        self.pos_lookup[(entity.depth, entity.x, entity.y)] = entity

    def add_entity(self, entity):
        self.entities.append(entity)
        self.pos_lookup[(entity.depth, entity.x, entity.y)] = entity
        self.iden_lookup[entity.iden] = entity

    def remove_entity(self, entity):
        del self.pos_lookup[(entity.depth, entity.x, entity.y)]
        del self.iden_lookup[entity.iden]
        self.entities.remove(entity)

    def view_for(self, entity: EntityView, reduce_tick: bool = False) -> "GameStateView":
        """GameState.view_for (state.py:53-58): the entity's depth only."""
        return GameStateView(False, self.tick - 1 if reduce_tick else self.tick,
                             self.world.shallow_copy_with_layers(entity.depth),
                             [e for e in self.entities if e.depth == entity.depth],
                             self.player_1_iden, self.player_2_iden)

    def view_spec(self) -> "GameStateView":
        return GameStateView(False, self.tick, self.world, self.entities, self.player_1_iden,
                             self.player_2_iden)

    def to_prims(self) -> bytes:
        """GameState.to_prims (state.py:94-112): auth byte, tick / player idens
        (big-endian u32), World (u64 length + bytes), entity count u32, then per
        entity u32 length + serializer.serialize(entity)."""
        w = self.world.to_prims()
        out = [struct.pack(">BIII", 1 if self.is_authoritative else 0, self.tick,
                           self.player_1_iden, self.player_2_iden),
               struct.pack(">Q", len(w)), w, struct.pack(">I", len(self.entities))]
        for e in self.entities:
            b = e.serialize()
            out.append(struct.pack(">I", len(b)))
            out.append(b)
        return b"".join(out)

    def serialize(self) -> bytes:
        """serializer.serialize(game_state): the JSON envelope with the a85 body
        (serializer.py:71-78, 134-156) -- what SyncPacket carries."""
        return _json({"iden": GAME_STATE_IDEN,
                      "prims": ascii85(self.to_prims()).decode("ascii")})

    def __eq__(self, other):  # GameState.__eq__ (state.py:134-152)
        return (isinstance(other, GameStateView)
                and self.is_authoritative == other.is_authoritative
                and self.tick == other.tick and self.player_1_iden == other.player_1_iden
                and self.player_2_iden == other.player_2_iden and self.world == other.world
                and self.entities == other.entities)


def world_depths(cfg, d1: int, d2: int) -> List[int]:
    """Depths of World.dungeons for players at (d1, d2), in insertion order.

    Unreachable despawn (updater.py:253-254): a depth exists iff some player
    has stood on it (start <= depth <= current) and not both players are
    deeper; Together starts create depths in increasing order, so that is the
    dict order.  Unused (:255-256): exactly the players' depths.  (For
    Separated starts the insertion order interleaves the two fronts by time;
    the set is exact, the order listed here is increasing.)"""
    sep = int(cfg.start_mode) == StartMode.Separated
    s1, s2 = (int(cfg.p1_depth), int(cfg.p2_depth)) if sep else (0, 0)
    if int(cfg.despawn) == DungeonDespawningStrategy.Unreachable:
        lo = min(d1, d2)
        return sorted(set(range(max(s1, lo), d1 + 1)) | set(range(max(s2, lo), d2 + 1)))
    return [d1] if d1 == d2 else [d1, d2]


def game_state(snap: dict, i: int, cfg, extra_stairs: Optional[Dict[int, tuple]] = None,
               bank=None) -> GameStateView:
    """Game ``i`` of a BatchedEngine.snapshot() in the reference schema.

    The world holds the players' current dungeons; with ``extra_stairs``
    ({depth: (sx, sy[, layout])}, from ``BatchedEngine.game_states``) it holds
    every dungeon of World.dungeons (``world_depths``).  With a dungeon bank
    (``bank``, snapshot with ``p_layout``) the dungeons are its layouts."""
    W, H = int(cfg.width), int(cfg.height)
    ents = []
    dungeons = {}
    cur = {}

    def view(sx, sy, lay=-1):
        if bank is not None:
            return DungeonView(W, H, sx, sy, tiles=bank.tiles(int(lay)))
        return DungeonView(W, H, sx, sy)

    rpg = snap.get("p_rpg")  # the character mechanics: items raise the base stats
    for p in range(2):
        d = int(snap["p_depth"][p][i])
        mhp, dmg = ((rpg[3][p][i], rpg[2][p][i]) if rpg is not None
                    else (cfg.player_health, cfg.player_damage))
        ents.append(EntityView(1 + p, d, snap["p_x"][p][i], snap["p_y"][p][i],
                               snap["p_health"][p][i], mhp, dmg, cfg.player_armor))
        lay = int(snap["p_layout"][p][i]) if bank is not None else -1
        cur.setdefault(d, (int(snap["st_x"][p][i]), int(snap["st_y"][p][i]), lay))
    if extra_stairs is None:
        for d, key in cur.items():
            dungeons[d] = view(*key)
    else:
        for d in world_depths(cfg, int(snap["p_depth"][0][i]), int(snap["p_depth"][1][i])):
            dungeons[d] = view(*(cur[d] if d in cur else extra_stairs[d]))
    K = int(cfg.n_npcs)
    if K:
        alive = np.asarray(snap["npc_alive"])
        alive = [int(v) for v in (alive[i:i + 1] if alive.ndim == 1 else alive[:, i])]
        npc_depth = int(cfg.p1_depth) if int(cfg.start_mode) == 2 else 0
        for k in range(K):
            if (alive[k // 32] >> (k % 32)) & 1:
                v = int(snap["npc_pos"][k][i])
                ents.append(EntityView(3 + k, npc_depth, v & 0xFF, v >> 8, snap["npc_health"][k][i],
                                       cfg.npc_health, cfg.npc_damage, cfg.npc_armor))
    return GameStateView(True, int(snap["tick"][i]), WorldView(dungeons), ents)


class BotDriver:
    """Drives batched games with per-game ``Bot`` objects (the reference's
    optimax_rogue_bots/bot.py interface): each step builds every game's
    ``view_for`` its bot's entity, calls ``bot.move`` and steps the engine;
    ``bot.finished`` is called when a game ends (optimax_rogue_bots/main.py:118-155).
    """

    def __init__(self, engine, bots_p1: Sequence, bots_p2: Sequence):
        if len(bots_p1) != engine.B or len(bots_p2) != engine.B:
            raise ValueError("one bot per game and player")
        self.engine = engine
        self.bots = (list(bots_p1), list(bots_p2))
        self._started = False

    def _views(self, snap):
        for i in range(self.engine.B):
            gs = game_state(snap, i, self.engine.cfg)
            yield i, gs

    def step(self) -> np.ndarray:
        import torch
        snap = self.engine.snapshot()
        acts = np.full((self.engine.B, 2), Move.Stay.value, np.int8)
        for i, gs in self._views(snap):
            for p in range(2):
                bot = self.bots[p][i]
                view = gs.view_for(gs.iden_lookup[1 + p])
                if not self._started:
                    bot.started(view)
                mv = bot.move(view)
                bot.on_move(view, mv)
                acts[i, p] = int(mv)
        self._started = True
        self.engine.actions.copy_(torch.from_numpy(acts))
        status = self.engine.step().cpu().numpy()
        done = np.nonzero((status >= UpdateResult.Player1Win) & (status <= UpdateResult.Tie)
                          & (snap["status"] == UpdateResult.InProgress))[0]
        if len(done):
            after = self.engine.snapshot()
            for i in done:
                gs = game_state(after, int(i), self.engine.cfg)
                for p in range(2):
                    self.bots[p][i].finished(gs.view_for(gs.iden_lookup[1 + p]),
                                             UpdateResult(int(status[i])))
        return status
