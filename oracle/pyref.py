"""TEST INFRASTRUCTURE ONLY -- a pure-Python object-model restatement of the
reference updater, for the CPU baseline beside the GPU number.

The reference itself cannot travel to the GPU box, so its cost profile is
restated here in the reference's own style: ``Entity`` objects in a list, a
``pos_lookup`` dict keyed by (depth, x, y), ``World`` as a {depth: Dungeon}
dict of numpy tile arrays, ``Dungeon.staircase`` as an ``np.argwhere`` scan,
``get_random_unblocked`` as the reference's arange / boolean-mask selection,
attribles recomputed by ``on_tick``, CPython's ``shuffle`` / ``choice``
semantics over the injected bits -- one game stepped per Python call, no
vectorization.  It is bit-exact against the reference's golden fixtures for
every reference-semantics case (tests/test_pyref.py), so it computes what the
reference computes, at the reference's kind of cost.  Only tests/ and
bench.py's cpu_baseline leg import it; the product package never does.

Restated (paths relative to the reference repository):
  Updater.update            optimax_rogue/logic/updater.py:76-162
  Updater.handle_move       optimax_rogue/logic/updater.py:180-243
  Updater.should_despawn    optimax_rogue/logic/updater.py:245-257
  Updater.handle_descend    optimax_rogue/logic/updater.py:259-296
  Updater.handle_combat     optimax_rogue/logic/updater.py:298-338
  calculate_pos             optimax_rogue/logic/updater.py:340-351
  Dungeon.is_blocked / staircase / get_random_unblocked
                            optimax_rogue/game/world.py:41-66
  EmptyDungeonGenerator.spawn_dungeon   optimax_rogue/logic/worldgen.py:33-43
  Together/SeparatedGameStartGenerator.setup_game  worldgen.py:77-87, 124-135
  GameState.move_entity / add_entity / remove_entity  game/state.py:64-88
  GameState.on_tick, Entity.on_tick, attribles  state.py:46-51,
                            entities.py:70-74, attribles.py:21-43
  RandomBot.move            optimax_rogue_bots/randombot.py:20-21
  StaircaseBot.move         optimax_rogue_bots/staircasebot.py:9-21

Random draws: the engine's keyed Philox4x32-10 streams at the reference's
draw sites exactly as tests/golden/make_golden.py injects them (DESIGN.md
s4; restated independently here), or -- stock-seed mode, cfg rng = 1 --
each game's own ``random.Random(n)`` / ``np.random.RandomState(n)``, n = seed
+ global game id, consumed in the reference's call order.

    python -m oracle.pyref --bench [--seconds S] [--procs N]   # CPU baseline JSON
"""
from __future__ import annotations

import json
import os
import random
import sys
import time

import numpy as np

M = 0xFFFFFFFF
PUR_INIT, PUR_DUNGEON, PUR_SHUFFLE, PUR_SPAWN, PUR_POLICY, PUR_TICK = 1, 2, 3, 4, 5, 7
PUR_NPC = 9   # the enemy AI's draws (npc_policy RANDOM, include/orx.h)
GROUND, WALL, STAIRS = 1, 2, 3                       # Tile (world.py:10-17)
UP, RIGHT, DOWN, LEFT, STAY = 1, 2, 3, 4, 5          # Move (moves.py:6-12)
MOVES = (UP, RIGHT, DOWN, LEFT, STAY)                # list(Move) (randombot.py:17-18)
BLOCK, AMBUSH, FLEE, PARRY = 1, 2, 3, 4              # CombatFlag (modifiers.py:7-12)
IN_PROGRESS, P1_WIN, P2_WIN, TIE = 1, 2, 3, 4        # UpdateResult (updater.py:16-21)
UNREACHABLE, UNUSED = 1, 2                           # DungeonDespawningStrategy (:47-50)
EV_COMBAT, EV_DEATH, EV_POSITION, EV_DUNGEON = 1, 2, 3, 4


# --------------------------------------------------------------------------
# random words
# --------------------------------------------------------------------------
def philox(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (Random123): 10 rounds of two 32x32->64 products."""
    for _ in range(10):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & M, p1 & M, ((p0 >> 32) ^ c3 ^ k1) & M, p0 & M
        k0 = (k0 + 0x9E3779B9) & M
        k1 = (k1 + 0xBB67AE85) & M
    return c0, c1, c2, c3


class Words:
    """Keyed whole-word stream: counter (game, episode, c2, purpose << 28 |
    gen << 24 | block), 4 words per block."""
    __slots__ = ("k0", "k1", "c0", "c1", "c2", "c3", "i", "buf")

    def __init__(self, seed, game, episode, c2, purpose, gen=0):
        self.k0, self.k1 = seed & M, (seed >> 32) & M
        self.c0, self.c1, self.c2 = game & M, episode & M, c2 & M
        self.c3 = (purpose << 28) | (gen << 24)
        self.i = 0
        self.buf = None

    def next(self):
        j = self.i & 3
        if j == 0:
            self.buf = philox(self.c0, self.c1, self.c2, self.c3 | (self.i >> 2), self.k0,
                              self.k1)
        self.i += 1
        return self.buf[j]

    def getrandbits(self, k):
        return self.next() >> (32 - k)


class TickBits:
    """A tick's CPython-random bits: reservoir segments of the
    TICK block -- word a for the updater's shuffles, bits 0-29 of words b
    then c for the bots -- least-significant bits first; a draw that does not
    fit the current segment skips it; past the last, the top k bits of the
    next word of the purpose's own stream."""
    __slots__ = ("segs", "fallback")

    def __init__(self, seed, game, episode, tick, purpose):
        w = philox(game & M, episode & M, tick & M, PUR_TICK << 28, seed & M, (seed >> 32) & M)
        self.segs = [[w[0], 32]] if purpose == PUR_SHUFFLE else \
            [[w[1] & 0x3FFFFFFF, 30], [w[2] & 0x3FFFFFFF, 30]]
        self.fallback = Words(seed, game, episode, tick, purpose)

    def getrandbits(self, k):
        segs = self.segs
        while segs and segs[0][1] < k:
            segs.pop(0)
        if not segs:
            return self.fallback.getrandbits(k)
        s = segs[0]
        r = s[0] & ((1 << k) - 1)
        s[0] >>= k
        s[1] -= k
        return r


class NpcBits:
    """The enemy AI's bits (npc_policy RANDOM): bits 0-29 of each successive
    word of the NPC stream as reservoir segments, least-significant first."""
    __slots__ = ("words", "seg", "n")

    def __init__(self, seed, game, episode, tick):
        self.words = Words(seed, game, episode, tick, PUR_NPC)
        self.seg, self.n = 0, 0

    def getrandbits(self, k):
        if self.n < k:
            self.seg, self.n = self.words.next() & 0x3FFFFFFF, 30
        r = self.seg & ((1 << k) - 1)
        self.seg >>= k
        self.n -= k
        return r


def randbelow(bits, n):
    """CPython Random._randbelow_with_getrandbits (Lib/random.py, 3.10)."""
    k = n.bit_length()
    r = bits.getrandbits(k)
    while r >= n:
        r = bits.getrandbits(k)
    return r


def shuffle(bits, x):
    """random.shuffle (Lib/random.py, 3.10) over a bit source."""
    for i in reversed(range(1, len(x))):
        j = randbelow(bits, i + 1)
        x[i], x[j] = x[j], x[i]


def np_randint(words, low, high=None):
    """numpy legacy RandomState.randint(low, high) for a scalar: masked
    rejection over 32-bit words (_bounded_integers.pyx, use_masked)."""
    if high is None:
        low, high = 0, low
    rng = high - 1 - low
    if rng == 0:
        return low
    mask = (1 << rng.bit_length()) - 1
    while True:
        v = words.next() & mask
        if v <= rng:
            return low + v


class StockPy:
    """The stock CPython random of one game: bits from random.Random(n)."""
    __slots__ = ("r",)

    def __init__(self, r):
        self.r = r

    def getrandbits(self, k):
        return self.r.getrandbits(k)


def stock_randint(rs, low, high=None):
    """numpy's own RandomState.randint (the stock reference's draw)."""
    return int(rs.randint(low, high)) if high is not None else int(rs.randint(low))


# --------------------------------------------------------------------------
# the game-state object model (game/world.py, game/entities.py, game/state.py)
# --------------------------------------------------------------------------
class Dungeon:
    __slots__ = ("tiles", "layout")

    def __init__(self, tiles, layout=-1):
        self.tiles = tiles
        self.layout = layout

    def is_blocked(self, x, y):
        t = self.tiles
        if x < 0 or x >= t.shape[0] or y < 0 or y >= t.shape[1]:
            return True
        return t[x, y] == WALL

    def staircase(self):
        x, y = tuple(np.argwhere(self.tiles == STAIRS)[0])
        return int(x), int(y)

    def get_random_unblocked(self, randint):
        avail = self.tiles == GROUND
        inds = np.arange(avail.shape[0] * avail.shape[1]).reshape(avail.shape)[avail]
        flat = inds[randint(inds.shape[0])]
        x = flat // avail.shape[1]
        y = flat - x * avail.shape[1]
        return int(x), int(y)


class Entity:
    __slots__ = ("iden", "depth", "x", "y", "health", "base_max_health", "base_damage",
                 "base_armor", "max_health", "damage", "armor")

    def __init__(self, iden, depth, x, y, health, base_max_health, base_damage, base_armor):
        self.iden, self.depth, self.x, self.y, self.health = iden, depth, x, y, health
        self.base_max_health, self.base_damage, self.base_armor = (base_max_health, base_damage,
                                                                   base_armor)
        self.max_health = self.damage = self.armor = None   # attribles: None until on_tick

    def on_tick(self):
        # attribles.py:21-43: base + sum of the (absent) modifiers' flat bonuses
        self.max_health = self.base_max_health + sum(())
        self.damage = self.base_damage + sum(())
        self.armor = self.base_armor + sum(())


class GameState:
    __slots__ = ("tick", "entities", "world", "pos_lookup", "iden_lookup")

    def __init__(self, tick, world, entities):
        self.tick = tick
        self.world = world
        self.entities = entities
        self.pos_lookup = {(e.depth, e.x, e.y): e for e in entities}
        self.iden_lookup = {e.iden: e for e in entities}

    def on_tick(self):
        for e in self.entities:
            e.on_tick()

    def move_entity(self, e, depth, x, y):
        del self.pos_lookup[(e.depth, e.x, e.y)]
        e.depth, e.x, e.y = depth, x, y
        self.pos_lookup[(depth, x, y)] = e

    def add_entity(self, e):
        self.entities.append(e)
        self.pos_lookup[(e.depth, e.x, e.y)] = e
        self.iden_lookup[e.iden] = e

    def remove_entity(self, e):
        del self.pos_lookup[(e.depth, e.x, e.y)]
        del self.iden_lookup[e.iden]
        self.entities.remove(e)


def calculate_pos(x, y, move):
    if move == UP:
        return x, y - 1
    if move == DOWN:
        return x, y + 1
    if move == RIGHT:
        return x + 1, y
    if move == LEFT:
        return x - 1, y
    return x, y


# --------------------------------------------------------------------------
# one game: generator, updater, bots and the harness around them
# --------------------------------------------------------------------------
class Game:
    """One reference game (GameState + Updater + two bots) with the engine's
    stream keys (or stock seeding); ``step`` autoresets like the engine."""

    def __init__(self, cfg, seed, gid, layouts=None):
        if cfg.get("flags", 0):
            raise ValueError("pyref restates the reference only (flags must be 0)")
        self.cfg, self.seed, self.gid = cfg, int(seed), int(gid)
        self.W, self.H = int(cfg["width"]), int(cfg["height"])
        self.layouts = None if layouts is None else np.asarray(layouts).astype(np.int32)
        self.max_ticks = int(cfg["max_ticks"]) or None
        self.stock = int(cfg.get("rng", 0)) == 1
        if self.stock:
            n = self.seed + self.gid
            self.py = StockPy(random.Random(n))
            self.np = np.random.RandomState(n)
        self.episode = 0
        self.status = IN_PROGRESS
        self.ret_sum = self.ep_count = 0
        self.counters = [0, 0, 0, 0]
        self.policy_codes = tuple(cfg.get("policy", (1, 1)))
        self.setup()

    # -- draws at the reference's sites -----------------------------------
    def _randint(self, words):
        if self.stock:
            return lambda lo, hi=None: stock_randint(self.np, lo, hi)
        return lambda lo, hi=None: np_randint(words, lo, hi)

    def spawn_dungeon(self, depth):
        """EmptyDungeonGenerator.spawn_dungeon, or a bank's randint(L) layout,
        from the (episode, depth, generation) stream."""
        gen = self.gens.get(depth, 0)
        self.gens[depth] = gen + 1
        ri = self._randint(Words(self.seed, self.gid, self.episode, depth, PUR_DUNGEON, gen))
        if self.layouts is not None:
            k = ri(len(self.layouts))
            return Dungeon(self.layouts[k].copy(), k)
        tiles = np.zeros((self.W, self.H), "int32")
        tiles[:, :] = GROUND
        tiles[[0, -1], :] = WALL
        tiles[:, [0, -1]] = WALL
        rx = ri(1, self.W - 2)
        ry = ri(1, self.H - 2)
        tiles[rx, ry] = STAIRS
        return Dungeon(tiles)

    def setup(self):
        """TogetherGameStartGenerator / SeparatedGameStartGenerator.setup_game
        and the NPC spawner (make_golden.NpcGameStart)."""
        c = self.cfg
        self.gens = {}
        ri = self._randint(Words(self.seed, self.gid, self.episode, 0, PUR_INIT))
        if int(c["start_mode"]) == 2:
            d1, d2 = int(c["p1_depth"]), int(c["p2_depth"])
            g1, g2 = self.spawn_dungeon(d1), self.spawn_dungeon(d2)
            x1, y1 = g1.get_random_unblocked(ri)
            x2, y2 = g2.get_random_unblocked(ri)
            world = {d1: g1, d2: g2}
        else:
            d1 = d2 = 0
            g1 = self.spawn_dungeon(0)
            x1, y1 = g1.get_random_unblocked(ri)
            x2, y2 = g1.get_random_unblocked(ri)
            while (x2, y2) == (x1, y1):
                x2, y2 = g1.get_random_unblocked(ri)
            world = {0: g1}
        ents = [Entity(1, d1, x1, y1, 10, 10, 2, 1), Entity(2, d2, x2, y2, 10, 10, 2, 1)]
        self.gs = gs = GameState(1, world, ents)
        hp, dmg, arm = int(c["npc_health"]), int(c["npc_damage"]), int(c["npc_armor"])
        for k in range(int(c["n_npcs"])):
            x, y = g1.get_random_unblocked(ri)
            while (d1, x, y) in gs.pos_lookup:
                x, y = g1.get_random_unblocked(ri)
            gs.add_entity(Entity(3 + k, d1, x, y, hp, hp, dmg, arm))
        self.status = IN_PROGRESS

    def policy(self, given=(STAY, STAY)):
        """RandomBot.move / StaircaseBot.move for both players (code 1 / 2;
        0 = the given action)."""
        gs = self.gs
        bits = self.py if self.stock else TickBits(self.seed, self.gid, self.episode, gs.tick,
                                                   PUR_POLICY)
        out = []
        for p, code in enumerate(self.policy_codes):
            if code == 1:
                out.append(MOVES[randbelow(bits, len(MOVES))])
            elif code == 2:
                me = gs.iden_lookup[p + 1]
                stx, sty = gs.world[me.depth].staircase()
                dx, dy = stx - me.x, sty - me.y
                if abs(dx) > abs(dy):
                    out.append(RIGHT if dx > 0 else LEFT)
                else:
                    out.append(DOWN if dy > 0 else UP)
            else:
                out.append(int(given[p]))
        return out

    def step(self, m1, m2):
        """One engine step: a finished game restarts (the next episode's setup),
        else on_tick + Updater.update.  Returns the tick's update events."""
        if self.status != IN_PROGRESS:
            if self.cfg.get("autoreset", 1):
                self.episode += 1
                self.setup()
            return []
        gs = self.gs
        gs.on_tick()
        if self.stock:
            self.bits, self.spawn_ri = self.py, self._randint(None)
        else:
            self.bits = TickBits(self.seed, self.gid, self.episode, gs.tick, PUR_SHUFFLE)
            self.spawn_ri = self._randint(Words(self.seed, self.gid, self.episode, gs.tick,
                                                PUR_SPAWN))
        ev = []
        self.status = s = self.update(gs, m1, m2, ev)
        if s == P1_WIN:
            self.ret_sum += 1
        elif s == P2_WIN:
            self.ret_sum -= 1
        if s != IN_PROGRESS:
            self.ep_count += 1
        return ev

    # -- Updater (logic/updater.py) -----------------------------------------
    def update(self, gs, m1, m2, ev):
        p1, p2 = gs.iden_lookup[1], gs.iden_lookup[2]
        x, y = calculate_pos(p1.x, p1.y, m1)
        if gs.world[p1.depth].is_blocked(x, y):
            m1 = STAY
        x, y = calculate_pos(p2.x, p2.y, m2)
        if gs.world[p2.depth].is_blocked(x, y):
            m2 = STAY
        upd = [[p1, m1], [p2, m2]]
        shuffle(self.bits, upd)
        ai = None
        if int(self.cfg.get("npc_policy", 0)) == 1:
            ai = self.py if self.stock else NpcBits(self.seed, self.gid, self.episode, gs.tick)
        npcs = [[e, self.decide_npc_move(gs, e, ai)] for e in gs.entities
                if e.iden not in (1, 2)]
        shuffle(self.bits, npcs)
        upd.extend(npcs)
        order = {u[0].iden: i for i, u in enumerate(upd)}
        for i, u in enumerate(upd):
            self.handle_move(gs, i, u, upd, order, ev)
        i = len(gs.entities) - 1
        while i >= 0:
            e = gs.entities[i]
            if e.health <= 0 and e.iden not in (1, 2):
                ev.append((EV_DEATH, e.iden, 0, 0))
                self.counters[3] += 1
                gs.remove_entity(e)
            i -= 1
        gs.tick += 1
        if p1.health <= 0:
            return TIE if p2.health <= 0 else P2_WIN
        if p2.health <= 0:
            return P1_WIN
        if self.max_ticks and gs.tick >= self.max_ticks:
            return TIE
        return IN_PROGRESS

    def decide_npc_move(self, gs, e, ai):
        """Updater.decide_npc_move (updater.py:165-178): Stay, or the enemy AI
        of make_golden.NpcAiUpdater (include/orx.h ORX_NPC_*)."""
        pol = int(self.cfg.get("npc_policy", 0))
        if pol == 0 or e.depth not in gs.world:
            return STAY
        d = gs.world[e.depth]
        here = [p for p in (gs.iden_lookup[1], gs.iden_lookup[2]) if p.depth == e.depth]
        W, H = d.tiles.shape
        for p in here:
            for m in (UP, RIGHT, DOWN, LEFT):
                x, y = calculate_pos(p.x, p.y, m)
                if 0 <= x < W and 0 <= y < H and d.tiles[x, y] == STAIRS:
                    return STAY
        if pol == 1:
            m = MOVES[randbelow(ai, len(MOVES))]
        else:
            if not here:
                return STAY
            t = min(here, key=lambda p: abs(p.x - e.x) + abs(p.y - e.y))
            dx, dy = t.x - e.x, t.y - e.y
            m = (RIGHT if dx > 0 else LEFT) if abs(dx) > abs(dy) else (DOWN if dy > 0 else UP)
        if d.is_blocked(*calculate_pos(e.x, e.y, m)):
            return STAY
        return m

    def handle_move(self, gs, i, u, upd, order, ev):
        e, move = u
        if move == STAY:
            return
        x, y = calculate_pos(e.x, e.y, move)
        at = gs.pos_lookup.get((e.depth, x, y))
        if at is None:
            if gs.world[e.depth].tiles[x, y] == STAIRS:
                self.handle_descend(gs, e, ev)
                return
            ev.append((EV_POSITION, e.iden, e.depth, (x & 0xFFFF) | (y << 16)))
            gs.move_entity(e, e.depth, x, y)
            return
        j = order[at.iden]
        amove = upd[j][1]
        if amove == STAY:
            self.handle_combat(e, at, BLOCK, ev)
            return
        if calculate_pos(at.x, at.y, amove) == (x, y):
            self.handle_combat(e, at, PARRY, ev)
            return
        self.handle_combat(e, at, AMBUSH if j < i else FLEE, ev)

    def should_despawn(self, gs, depth):
        d1, d2 = gs.iden_lookup[1].depth, gs.iden_lookup[2].depth
        strat = int(self.cfg["despawn"])
        if strat == UNREACHABLE:
            return d1 > depth and d2 > depth
        if strat == UNUSED:
            return depth not in (d1, d2)
        raise ValueError(f"Unknown despawn strat {strat}")

    def handle_descend(self, gs, e, ev):
        if e.iden not in (1, 2):
            ev.append((EV_DEATH, e.iden, 0, 0))
            self.counters[3] += 1
            gs.remove_entity(e)
            return
        old = e.depth
        nd = old + 1
        if nd not in gs.world:
            gs.world[nd] = self.spawn_dungeon(nd)
            ev.append((EV_DUNGEON, 0, nd, 0))
            self.counters[2] += 1
        dung = gs.world[nd]
        x, y = dung.get_random_unblocked(self.spawn_ri)
        while (nd, x, y) in gs.pos_lookup:
            x, y = dung.get_random_unblocked(self.spawn_ri)
        ev.append((EV_POSITION, e.iden, nd, (x & 0xFFFF) | (y << 16)))
        self.counters[1] += 1
        gs.move_entity(e, nd, x, y)
        if self.should_despawn(gs, old):
            del gs.world[old]

    def handle_combat(self, att, dfn, flag, ev):
        dmg = att.damage - att.armor
        if dmg > 0:
            dfn.health -= dmg
        ev.append((EV_COMBAT, att.iden, dfn.iden, flag))
        self.counters[0] += 1

    # -- the engine's state row of this game ----------------------------------
    def snapshot(self):
        gs = self.gs
        p = (gs.iden_lookup[1], gs.iden_lookup[2])
        st = [gs.world[e.depth].staircase() for e in p]
        K = int(self.cfg["n_npcs"])
        pos, hp, alive = [0] * K, [0] * K, 0
        for e in gs.entities:
            if e.iden >= 3:
                k = e.iden - 3
                alive |= 1 << k
                pos[k] = (e.x & 0xFF) | ((e.y & 0xFF) << 8)
                hp[k] = e.health
        rec = {"p_x": [e.x for e in p], "p_y": [e.y for e in p],
               "p_depth": [e.depth for e in p], "p_health": [e.health for e in p],
               "st_x": [s[0] for s in st], "st_y": [s[1] for s in st], "tick": gs.tick,
               "status": self.status, "episode": self.episode, "ret_sum": self.ret_sum,
               "ep_count": self.ep_count, "counters": list(self.counters),
               "npc_pos": pos, "npc_health": hp,
               "npc_alive": alive if K <= 32 else [(alive >> (32 * w)) & M
                                                   for w in range((K + 31) // 32)]}
        if self.layouts is not None:
            rec["p_layout"] = [gs.world[e.depth].layout for e in p]
        return rec

    def world_list(self):
        w = self.gs.world
        if self.layouts is None:
            return [(d, *w[d].staircase()) for d in w]
        return [(d, *w[d].staircase(), w[d].layout) for d in w]

    def entity_list(self):
        return [(e.iden, e.depth, e.x, e.y, e.health) for e in self.gs.entities]


def batch_state(games):
    """Engine-layout SoA arrays ([2][B] players, [B] scalars, [4][B] counters,
    [K][B] NPC rows) of a list of games."""
    recs = [g.snapshot() for g in games]
    out = {}
    for k in recs[0]:
        a = np.array([r[k] for r in recs])
        out[k] = a.T if a.ndim == 2 else a
    return out


# --------------------------------------------------------------------------
# CPU baseline (bench.py's cpu_baseline leg): the C3 workload on host cores
# --------------------------------------------------------------------------
C3 = dict(width=64, height=64, despawn=1, max_ticks=1000, start_mode=1, p1_depth=0, p2_depth=0,
          n_npcs=8, npc_health=3, npc_damage=1, npc_armor=0, player_health=10, player_damage=2,
          player_armor=1, autoreset=1, flags=0, rng=0, policy=(1, 1))


def _leg(args):
    """One process: 16 C3 games (disjoint global ids) stepped round-robin with
    both RandomBots for `seconds`; returns (env-steps, seconds)."""
    k, seconds = args
    games = [Game(C3, 3, k * 16 + g) for g in range(16)]
    n = 0
    t0 = time.perf_counter()
    while True:
        for g in games:
            m1, m2 = g.policy()
            g.step(m1, m2)
        n += len(games)
        if n % 256 == 0 and time.perf_counter() - t0 >= seconds:
            break
    return n, time.perf_counter() - t0


def _lscpu():
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        keep = ("Model name", "CPU(s)", "Thread(s) per core", "Core(s) per socket", "Socket(s)",
                "CPU max MHz", "NUMA node(s)")
        return {k.strip(): v.strip() for k, v in (l.split(":", 1) for l in out.splitlines()
                                                  if ":" in l) if k.strip() in keep}
    except Exception as e:   # lscpu absent: the model from /proc/cpuinfo
        return {"error": str(e)}


def bench(seconds: float = 2.0, procs: int = 0, single_seconds: float = 3.0) -> dict:
    """Per-core (one process alone) and aggregate (one process per core of this
    job's CPU share, at most 16) env-steps/s of this restatement on C3."""
    import multiprocessing as mp
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    procs = procs or max(1, min(16, avail))
    n1, t1 = _leg((0, single_seconds))
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(procs) as pool:
        res = pool.map(_leg, [(k + 1, seconds) for k in range(procs)])
    wall = time.perf_counter() - t0
    total = sum(n for n, _ in res)
    return {"value": total / max(t for _, t in res), "unit": "env-steps/s", "cores": procs,
            "per_core": total / sum(t for _, t in res), "single_core": n1 / t1,
            "kind": "python_restatement",
            "sample": (f"pure-Python object-model restatement of the reference updater + 2x "
                       f"RandomBot (oracle/pyref.py, bit-exact vs the reference fixtures) on "
                       f"C3 (64x64, 8 NPCs, Unreachable, max_ticks 1000, autoreset): 1 process "
                       f"alone for {t1:.1f} s ({n1} env-steps), then {procs} processes x 16 "
                       f"games for {seconds:.1f} s each ({total} env-steps, {wall:.1f} s wall)"),
            "lscpu": _lscpu(), "cpus_visible": os.cpu_count(), "cpus_in_affinity": avail}


if __name__ == "__main__":
    if "--bench" in sys.argv:
        opts = dict(a[2:].split("=") for a in sys.argv[1:] if a.startswith("--") and "=" in a)
        print(json.dumps(bench(float(opts.get("seconds", 2.0)), int(opts.get("procs", 0)),
                               float(opts.get("single", 3.0)))), flush=True)
