"""Generates the golden fixtures in tests/golden/ from the REFERENCE updater.

Run in the build container only (it needs /root/reference; nothing at test
time imports the reference):

    python tests/golden/make_golden.py

What it does
------------
It imports the unmodified reference packages (optimax_rogue, optimax_rogue_bots)
and drives the in-process loop of SURVEY.md s3.3:
``gs.on_tick(); result, updates = Updater.update(gs, m1, m2)``
with the engine's Philox4x32-10 word stream injected at the reference's own draw
sites, so that the reference's code -- not a restatement -- computes every
output:

* ``optimax_rogue.logic.updater.random`` and ``optimax_rogue_bots.randombot.random``
  are replaced by a ``random.Random`` subclass whose ``getrandbits(k)`` returns
  the next k bits of the tick's reservoir, then ``word >> (32 - k)``.  CPython's own ``shuffle``/``choice``/``_randbelow``
  (Lib/random.py, 3.10) run unchanged on top of it (updater.py:114,127,
  randombot.py:21).
* ``np`` in ``optimax_rogue.logic.worldgen`` and ``optimax_rogue.game.world`` is
  a proxy whose ``random.randint`` is numpy's legacy bounded-integer transform
  (masked rejection over 32-bit words, numpy/random/_bounded_integers.pyx,
  ``_rand_int64`` -> ``random_bounded_uint64_fill`` with ``use_masked``);
  every other attribute is numpy itself (worldgen.py:39-40, world.py:62).
* Dungeons come from ``KeyedDungeonGenerator``, a subclass of the reference's
  ``EmptyDungeonGenerator`` (its plugin API, worldgen.py:9-43) that only selects
  the word stream (episode, depth, generation) before calling the reference's
  ``spawn_dungeon``.
* Explicit-grid cases (``layouts``): ``KeyedBankGenerator``, a subclass of the
  reference's ``DungeonGenerator`` (worldgen.py:9-26), returns the reference's
  ``Dungeon(tiles)`` for layout ``np.random.randint(L)`` of a fixed bank --
  the engine's dungeon-bank plugin; the reference's own ``is_blocked``,
  ``get_random_unblocked``, ``staircase`` and ``handle_move`` then run on
  walls, open borders and several staircases.  The bank is saved with the
  fixture.
* Stock-seed cases (``rng=1``) inject nothing: every game is a reference
  process of its own seeded with ``random.seed(n)`` and ``np.random.seed(n)``
  (n = seed + global game id) -- the module-level CPython ``random`` and numpy
  ``RandomState`` run unmodified (their states are swapped in and out per
  game), dungeons come from the stock ``EmptyDungeonGenerator``.  The
  engine's ORX_RNG_MT19937 mode must reproduce them from the seed alone.
* NPCs ("enemies") come from ``NpcGameStart``, a ``GameStartGenerator``
  (worldgen.py:47-58) that calls the reference's Together/Separated
  ``setup_game`` and then places K NPCs with the reference's
  ``Dungeon.get_random_unblocked`` and ``GameState.add_entity``.
* Moving NPCs (``npc_policy`` 1 / 2): ``NpcAiUpdater``, a subclass of the
  reference's ``Updater`` that overrides only its enemy-AI hook
  ``decide_npc_move`` (updater.py:165-178) -- the reference's ``update`` then
  draws the NPC shuffle, resolves every NPC move through ``handle_move`` /
  ``handle_combat`` / ``handle_descend`` (updater.py:116-145, 180-338) and
  sweeps the dead.  The AI (include/orx.h ORX_NPC_*): an NPC on a depth
  with no dungeon, or on a depth where a player stands next to a staircase,
  stays; otherwise RANDOM = ``random.choice(list(Move))`` (the updater's
  module ``random``, its words from the NPC stream ``NpcBits`` in keyed
  mode, the game's own CPython state in stock mode) and CHASE = a greedy step
  toward the nearer player on its depth (StaircaseBot's rule, player 1 on a
  tie); a move into a blocked cell becomes Stay (``Dungeon.is_blocked``).
  The staircase rule keeps the reference from raising: ``update`` asks
  every NPC's move before any move is made, and an NPC stepping onto a free
  cell of a depth that a player's descend despawned earlier in the same tick
  would hit ``World.get_at_depth``'s KeyError (updater.py:203, :295-296).

The third-party module ``inflection`` (imported by serializer.py:27, unpinned:
setup.py:11 has install_requires=[]) is not installed.  It is only used for
serializer registry names (serializer.py:95), never on the tick path; a stub
restating ``inflection.underscore`` (inflection 0.5.1: two regex passes, '-'
to '_', lower-case) is put in sys.modules.

Stream keys (must match include/orx.h / DESIGN.md): Philox key = seed;
counter = (global game id, episode, c2, purpose << 28 | gen << 24 | block)
with purposes INIT=1 (c2 = 0), DUNGEON=2 (c2 = depth), SHUFFLE=3, SPAWN=4,
POLICY=5, TICK=7 (c2 = tick before the update).  The CPython-random draws of a
tick (bots, shuffles) come from the TICK block's bit reservoir first
(``TickBits``).
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import random
import re
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

# --------------------------------------------------------------------------
# Philox4x32-10 (independent pure-Python implementation)
# --------------------------------------------------------------------------
M = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for _ in range(10):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & M, p1 & M, ((p0 >> 32) ^ c3 ^ k1) & M, p0 & M
        k0 = (k0 + 0x9E3779B9) & M
        k1 = (k1 + 0xBB67AE85) & M
    return c0, c1, c2, c3


PUR_INIT, PUR_DUNGEON, PUR_SHUFFLE, PUR_SPAWN, PUR_POLICY = 1, 2, 3, 4, 5
PUR_TICK = 7
PUR_NPC = 9   # the enemy AI's draws (c2 = tick): decide_npc_move's random.choice


class Stream:
    def __init__(self, seed, game, episode, c2, purpose, gen=0):
        self.key = (seed & M, (seed >> 32) & M)
        self.c = (game & M, episode & M, c2 & M, (purpose << 28) | (gen << 24))
        self.idx = 0
        self.buf = None

    def next(self):
        if self.idx % 4 == 0:
            self.buf = philox4x32_10(
                (self.c[0], self.c[1], self.c[2], self.c[3] | (self.idx // 4)), self.key)
        w = self.buf[self.idx % 4]
        self.idx += 1
        return w

    def getrandbits(self, k):
        return self.next() >> (32 - k)


class TickBits:
    """The bit source of one tick's CPython-random draws: the
    tick block Philox(game, episode, tick, TICK << 28) holds reservoir
    segments -- word 0 (32 bits) for the updater's shuffles; bits 0-29 of
    word 1, then bits 0-29 of word 2 for the bots -- consumed
    least-significant bits first.  A getrandbits(k) skips a segment with
    fewer than k bits left; once none is left it takes the top k bits of the
    next word of the purpose's own stream."""

    def __init__(self, seed, game, episode, tick, purpose):
        w = philox4x32_10((game & M, episode & M, tick & M, PUR_TICK << 28),
                          (seed & M, (seed >> 32) & M))
        if purpose == PUR_SHUFFLE:
            self.segs = [[w[0], 32]]
        else:
            self.segs = [[w[1] & 0x3FFFFFFF, 30], [w[2] & 0x3FFFFFFF, 30]]
        self.words = Stream(seed, game, episode, tick, purpose)

    def getrandbits(self, k):
        while self.segs and self.segs[0][1] < k:
            self.segs.pop(0)
        if not self.segs:
            return self.words.getrandbits(k)
        seg = self.segs[0]
        r = seg[0] & ((1 << k) - 1)
        seg[0] >>= k
        seg[1] -= k
        return r


class NpcBits:
    """The bit source of one tick's enemy-AI draws (npc_policy RANDOM): the
    stream (game, episode, tick, NPC << 28) taken as consecutive 30-bit
    reservoir segments -- bits 0-29 of word 0, of word 1, ... (four words a
    block) -- consumed least-significant bits first; a getrandbits(k) skips
    a segment with fewer than k bits left.  random.choice(list(Move)) takes
    3-bit fields: ten per word, a field >= 5 rejected (_randbelow)."""

    def __init__(self, seed, game, episode, tick):
        self.words = Stream(seed, game, episode, tick, PUR_NPC)
        self.seg = [0, 0]

    def getrandbits(self, k):
        assert k <= 30
        if self.seg[1] < k:
            self.seg = [self.words.next() & 0x3FFFFFFF, 30]
        r = self.seg[0] & ((1 << k) - 1)
        self.seg[0] >>= k
        self.seg[1] -= k
        return r


def philox_np(c0, c1, c2, c3, key):
    """Vectorized Philox4x32-10 over uint32 counter arrays (numpy uint64 math)."""
    c = [np.asarray(v, np.uint64) & M for v in (c0, c1, c2, c3)]
    k0, k1 = key
    for _ in range(10):
        p0 = c[0] * np.uint64(0xD2511F53)
        p1 = c[2] * np.uint64(0xCD9E8D57)
        c = [(p1 >> np.uint64(32)) ^ c[1] ^ np.uint64(k0), p1 & np.uint64(M),
             (p0 >> np.uint64(32)) ^ c[3] ^ np.uint64(k1), p0 & np.uint64(M)]
        k0 = (k0 + 0x9E3779B9) & M
        k1 = (k1 + 0xBB67AE85) & M
    return c


def find_reservoir_overflow(seed, episode, tick, kind, chunk=1 << 22):
    """First global game id whose tick block cannot serve the tick's draws:
    kind "shuffle" = all 16 two-bit fields of word 0 rejected (2^-16);
    "policy" = fewer than two of the 20 three-bit fields in bits 0-29 of
    words 1 and 2 accepted (~1e-7).  Those games exercise the fallback word streams."""
    key = (seed & M, (seed >> 32) & M)
    for start in range(0, 1 << 32, chunk):
        g = np.arange(start, start + chunk, dtype=np.uint64)
        w = philox_np(g, episode, tick, PUR_TICK << 28, key)
        if kind == "shuffle":
            bad = (~(w[0] >> np.uint64(1)) & np.uint64(0x55555555)) == 0
        else:
            n = np.zeros(len(g), np.int64)
            for v in (w[1], w[2]):
                rej = (v >> np.uint64(2)) & (v | (v >> np.uint64(1)))
                acc = ~rej & np.uint64(0x09249249)
                for j in range(10):
                    n += ((acc >> np.uint64(3 * j)) & np.uint64(1)).astype(np.int64)
            bad = n < 2
        hit = np.flatnonzero(bad)
        if len(hit):
            return int(g[hit[0]])
    raise RuntimeError("no overflow found")


class PhiloxRandom(random.Random):
    """random.Random whose bits come from the current Philox stream."""

    def __init__(self):
        super().__init__(0)
        self.stream = None

    def getrandbits(self, k):
        assert 0 < k <= 32
        return self.stream.getrandbits(k)


class NpRandom:
    """numpy.random stand-in exposing the legacy scalar randint transform."""

    def __init__(self):
        self.stream = None

    def randint(self, low, high=None, size=None, dtype=int):
        assert size is None
        if high is None:
            low, high = 0, low
        if low >= high:
            raise ValueError("low >= high")
        rng = high - 1 - low
        if rng == 0:
            return low
        mask = (1 << rng.bit_length()) - 1
        while True:
            v = self.stream.next() & mask
            if v <= rng:
                return low + v


class NpProxy:
    def __init__(self, rnd):
        self.random = rnd

    def __getattr__(self, name):
        return getattr(np, name)


def _underscore(word):
    word = re.sub(r"([A-Z]+)([A-Z][a-z])", r"\1_\2", word)
    word = re.sub(r"([a-z\d])([A-Z])", r"\1_\2", word)
    word = word.replace("-", "_")
    return word.lower()


def import_reference():
    stub = types.ModuleType("inflection")
    stub.underscore = _underscore
    sys.modules.setdefault("inflection", stub)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import optimax_rogue.logic.updater as updater_mod
    import optimax_rogue.logic.worldgen as worldgen_mod
    import optimax_rogue.game.world as world_mod
    import optimax_rogue_bots.randombot as randombot_mod
    import optimax_rogue_bots.staircasebot as staircasebot_mod
    import optimax_rogue.game.state as state_mod
    import optimax_rogue.game.entities as entities_mod
    import optimax_rogue.logic.updates as updates_mod
    import optimax_rogue.logic.moves as moves_mod
    pyrand = PhiloxRandom()
    nprand = NpRandom()
    updater_mod.random = pyrand
    randombot_mod.random = pyrand
    worldgen_mod.np = NpProxy(nprand)
    world_mod.np = NpProxy(nprand)
    return types.SimpleNamespace(
        updater=updater_mod, worldgen=worldgen_mod, world=world_mod,
        randombot=randombot_mod, staircasebot=staircasebot_mod, state=state_mod,
        entities=entities_mod, updates=updates_mod, moves=moves_mod,
        pyrand=pyrand, nprand=nprand, injected=(pyrand, NpProxy(nprand)))


@contextlib.contextmanager
def stock_rng(R, h):
    """Runs reference code with the real module-level random / np.random
    holding game h's own states (a separate seeded process per game)."""
    mods_py = (R.updater, R.randombot)
    mods_np = (R.worldgen, R.world)
    saved = [m.random for m in mods_py], [m.np for m in mods_np]
    for m in mods_py:
        m.random = random
    for m in mods_np:
        m.np = np
    random.setstate(h.py_state)
    np.random.set_state(h.np_state)
    try:
        yield
    finally:
        h.py_state = random.getstate()
        h.np_state = np.random.get_state()
        for m, v in zip(mods_py, saved[0]):
            m.random = v
        for m, v in zip(mods_np, saved[1]):
            m.np = v


# --------------------------------------------------------------------------
# Harness around the reference
# --------------------------------------------------------------------------
class Harness:
    """One reference game (GameState + Updater) with keyed streams."""

    def __init__(self, R, cfg, seed, game_id):
        self.R, self.cfg, self.seed, self.gid = R, cfg, seed, game_id
        self.episode = 0
        self.gens = {}
        self.stock = cfg.get("rng", 0) == 1
        if self.stock:
            n = seed + game_id
            self.py_state = random.Random(n).getstate()
            self.np_state = np.random.RandomState(n).get_state()
        R_ = R

        harness = self

        class KeyedDungeonGenerator(R_.worldgen.EmptyDungeonGenerator):
            def spawn_dungeon(self, depth):
                gen = harness.gens.get(depth, 0)
                harness.gens[depth] = gen + 1
                saved = R_.nprand.stream
                R_.nprand.stream = Stream(harness.seed, harness.gid, harness.episode, depth,
                                          PUR_DUNGEON, gen)
                try:
                    return super().spawn_dungeon(depth)
                finally:
                    R_.nprand.stream = saved

        class NpcGameStart(R_.worldgen.GameStartGenerator):
            def __init__(self, inner, k, hp, dmg, arm):
                self.inner, self.k, self.hp, self.dmg, self.arm = inner, k, hp, dmg, arm

            def setup_game(self):
                gs = self.inner.setup_game()
                d = gs.player_1.depth
                dung = gs.world.get_at_depth(d)
                for k in range(self.k):
                    x, y = dung.get_random_unblocked()
                    while (d, x, y) in gs.pos_lookup:
                        x, y = dung.get_random_unblocked()
                    gs.add_entity(R_.entities.Entity(3 + k, d, x, y, self.hp, self.hp,
                                                     self.dmg, self.arm, [], dict()))
                return gs

        class KeyedBankGenerator(R_.worldgen.DungeonGenerator):
            def __init__(self, width, height, layouts):
                super().__init__(width, height)
                self.layouts = layouts

            def spawn_dungeon(self, depth):
                gen = harness.gens.get(depth, 0)
                harness.gens[depth] = gen + 1
                saved = R_.nprand.stream
                R_.nprand.stream = Stream(harness.seed, harness.gid, harness.episode, depth,
                                          PUR_DUNGEON, gen)
                try:
                    idx = R_.worldgen.np.random.randint(len(self.layouts))
                finally:
                    R_.nprand.stream = saved
                return R_.world.Dungeon(self.layouts[idx].astype(np.int32))

        class StockBankGenerator(R_.worldgen.DungeonGenerator):
            def __init__(self, width, height, layouts):
                super().__init__(width, height)
                self.layouts = layouts

            def spawn_dungeon(self, depth):
                idx = R_.worldgen.np.random.randint(len(self.layouts))
                return R_.world.Dungeon(self.layouts[idx].astype(np.int32))

        self.layouts = cfg.get("layouts")
        if self.stock:
            self.dgen = (StockBankGenerator(cfg["width"], cfg["height"], self.layouts)
                         if self.layouts is not None
                         else R_.worldgen.EmptyDungeonGenerator(cfg["width"], cfg["height"]))
        elif self.layouts is not None:
            self.dgen = KeyedBankGenerator(cfg["width"], cfg["height"], self.layouts)
        else:
            self.dgen = KeyedDungeonGenerator(cfg["width"], cfg["height"])
        if cfg["start_mode"] == 2:
            inner = R.worldgen.SeparatedGameStartGenerator(self.dgen, cfg["p1_depth"],
                                                           cfg["p2_depth"])
        else:
            inner = R.worldgen.TogetherGameStartGenerator(self.dgen)
        self.start = NpcGameStart(inner, cfg["n_npcs"], cfg["npc_health"], cfg["npc_damage"],
                                  cfg["npc_armor"])
        Move = R.moves.Move

        def next_to_stairs(dung, p):
            for m in (Move.Up, Move.Right, Move.Down, Move.Left):
                x, y = R_.updater.calculate_pos(p.x, p.y, m)
                if 0 <= x < dung.width and 0 <= y < dung.height \
                        and dung.tiles[x, y] == R_.world.Tile.StaircaseDown:
                    return True
            return False

        class NpcAiUpdater(R_.updater.Updater):
            """The reference's Updater with its enemy-AI hook overridden
            (updater.py:165-178); nothing else of it is touched."""

            def decide_npc_move(self, game_state, ent, result):
                if ent.depth not in game_state.world.dungeons:
                    return Move.Stay
                dung = game_state.world.get_at_depth(ent.depth)
                players = [p for p in (game_state.player_1, game_state.player_2)
                           if p.depth == ent.depth]
                if any(next_to_stairs(dung, p) for p in players):
                    return Move.Stay
                if harness.npc_policy == 1:      # RANDOM
                    saved = R_.pyrand.stream
                    if not harness.stock:
                        R_.pyrand.stream = harness.npc_bits
                    try:
                        move = R_.updater.random.choice(list(Move))
                    finally:
                        R_.pyrand.stream = saved
                else:                           # CHASE
                    if not players:
                        return Move.Stay
                    tgt = min(players, key=lambda p: abs(p.x - ent.x) + abs(p.y - ent.y))
                    dx, dy = tgt.x - ent.x, tgt.y - ent.y
                    if abs(dx) > abs(dy):
                        move = Move.Right if dx > 0 else Move.Left
                    else:
                        move = Move.Down if dy > 0 else Move.Up
                if dung.is_blocked(*R_.updater.calculate_pos(ent.x, ent.y, move)):
                    return Move.Stay
                return move

        self.npc_policy = int(cfg.get("npc_policy", 0))
        self.npc_bits = None
        strat = R.updater.DungeonDespawningStrategy(cfg["despawn"])
        upd_cls = NpcAiUpdater if self.npc_policy else R.updater.Updater
        self.updater = upd_cls(self.dgen, strat, cfg["max_ticks"] or None)
        self.bots = [self._bot(cfg["policy"][0], 1), self._bot(cfg["policy"][1], 2)]
        self.ret_sum = 0
        self.ep_count = 0
        self.counters = [0, 0, 0, 0]
        self.status = 1
        self.setup()

    def _bot(self, pol, iden):
        if pol == 1:
            return self.R.randombot.RandomBot(iden)
        if pol == 2:
            return self.R.staircasebot.StaircaseBot(iden)
        return None

    def setup(self):
        self.gens = {}
        if self.stock:
            with stock_rng(self.R, self):
                self.gs = self.start.setup_game()
        else:
            self.R.nprand.stream = Stream(self.seed, self.gid, self.episode, 0, PUR_INIT)
            self.gs = self.start.setup_game()
        self.status = 1

    def policy(self, given=None):
        if self.stock:
            with stock_rng(self.R, self):
                return self._policy(given)
        self.R.pyrand.stream = TickBits(self.seed, self.gid, self.episode, self.gs.tick, PUR_POLICY)
        return self._policy(given)

    def _policy(self, given):
        acts = []
        for p in range(2):
            bot = self.bots[p]
            if bot is None:
                acts.append(int(given[p]))
            else:
                acts.append(int(bot.move(self.gs)))
        return acts

    def step(self, acts):
        """One engine step: autoreset a finished game, else one reference tick."""
        R = self.R
        events = []
        if self.status != 1:
            if self.cfg["autoreset"]:
                self.episode += 1
                self.setup()
            return events
        self.gs.on_tick()
        if self.stock:
            with stock_rng(R, self), contextlib.redirect_stdout(io.StringIO()):
                res, upds = self.updater.update(self.gs, R.moves.Move(acts[0]),
                                                R.moves.Move(acts[1]))
        else:
            R.pyrand.stream = TickBits(self.seed, self.gid, self.episode, self.gs.tick, PUR_SHUFFLE)
            R.nprand.stream = Stream(self.seed, self.gid, self.episode, self.gs.tick, PUR_SPAWN)
            self.npc_bits = NpcBits(self.seed, self.gid, self.episode, self.gs.tick)
            with contextlib.redirect_stdout(io.StringIO()):
                res, upds = self.updater.update(self.gs, R.moves.Move(acts[0]),
                                                R.moves.Move(acts[1]))
        self.status = int(res)
        if self.status == 2:
            self.ret_sum += 1
        elif self.status == 3:
            self.ret_sum -= 1
        if self.status != 1:
            self.ep_count += 1
        U = R.updates
        for u in upds:
            if isinstance(u, U.EntityCombatUpdate):
                (flag,) = tuple(u.tags)
                events.append((1, u.attacker_iden, u.defender_iden, int(flag)))
                self.counters[0] += 1
            elif isinstance(u, U.EntityDeathUpdate):
                events.append((2, u.entity_iden, 0, 0))
                if u.entity_iden not in (1, 2):
                    self.counters[3] += 1
            elif isinstance(u, U.EntityPositionUpdate):
                events.append((3, u.entity_iden, u.depth, (u.posx & 0xFFFF) | (u.posy << 16)))
                if u.depth != u.old_depth:
                    self.counters[1] += 1
            elif isinstance(u, U.DungeonCreatedUpdate):
                events.append((4, 0, u.depth, 0))
                self.counters[2] += 1
            else:
                raise AssertionError(type(u))
        return events

    def snapshot(self):
        gs = self.gs
        K = self.cfg["n_npcs"]
        p = [gs.player_1, gs.player_2]
        rec = {}
        rec["p_x"] = [e.x for e in p]
        rec["p_y"] = [e.y for e in p]
        rec["p_depth"] = [e.depth for e in p]
        rec["p_health"] = [e.health for e in p]
        st = [gs.world.get_at_depth(e.depth).staircase() for e in p]
        rec["st_x"] = [s[0] for s in st]
        rec["st_y"] = [s[1] for s in st]
        rec["tick"] = gs.tick
        rec["status"] = self.status
        rec["episode"] = self.episode
        rec["ret_sum"] = self.ret_sum
        rec["ep_count"] = self.ep_count
        rec["counters"] = list(self.counters)
        pos = [0] * K
        hp = [0] * K
        alive = 0
        for e in gs.entities:
            if e.iden >= 3:
                k = e.iden - 3
                alive |= 1 << k
                pos[k] = (e.x & 0xFF) | ((e.y & 0xFF) << 8)
                hp[k] = e.health
        rec["npc_pos"] = pos
        rec["npc_health"] = hp
        # one 32-bit word per game up to 32 NPCs (the committed fixtures), rows
        # of 32 alive bits beyond (the engine's dense layout, [words][games])
        rec["npc_alive"] = alive if K <= 32 else [(alive >> (32 * w)) & 0xFFFFFFFF
                                                  for w in range((K + 31) // 32)]
        if self.layouts is None:
            rec["world"] = [(d, *gs.world.dungeons[d].staircase()) for d in gs.world.dungeons]
        else:
            lay = lambda dung: next(i for i, t in enumerate(self.layouts)
                                    if np.array_equal(dung.tiles, t))
            rec["world"] = [(d, *gs.world.dungeons[d].staircase(), lay(gs.world.dungeons[d]))
                            for d in gs.world.dungeons]
            rec["p_layout"] = [lay(gs.world.get_at_depth(e.depth)) for e in p]
        rec["entities"] = [(e.iden, e.depth, e.x, e.y, e.health) for e in gs.entities]
        return rec


def make_layouts(W, H, L, seed, n_stairs=(1,), open_border=False, wall_p=0.18):
    """A deterministic bank of L layouts (Tile codes, [L, W, H]): border walls
    (with gaps when open_border), random interior walls, n_stairs[l] staircases."""
    rs = np.random.RandomState(seed)
    out = []
    for li in range(L):
        t = np.ones((W, H), np.uint8)
        t[[0, -1], :] = 2
        t[:, [0, -1]] = 2
        if open_border and li % 2 == 0:  # Ground on the edge: moving off it is out of bounds
            t[0, 1:H - 1] = 1
            t[1:W - 1, H - 1] = 1
        inner = rs.rand(W, H) < wall_p
        inner[[0, -1], :] = False
        inner[:, [0, -1]] = False
        t[inner] = 2
        ground = np.argwhere(t == 1)
        pick = rs.choice(len(ground), n_stairs[li % len(n_stairs)], replace=False)
        for j in pick:
            t[tuple(ground[j])] = 3
        out.append(t)
    return np.stack(out)


DEFAULT_CFG = dict(width=32, height=32, despawn=1, max_ticks=1000, start_mode=1, p1_depth=0,
                   p2_depth=0, n_npcs=0, npc_health=3, npc_damage=1, npc_armor=0,
                   player_health=10, player_damage=2, player_armor=1, autoreset=1, flags=0,
                   policy=(1, 1), npc_policy=0)

CASES = {
    # C1 of BASELINE.json: 32x32, 2x RandomBot, max_ticks 1000 (long enough to autoreset)
    "c1_random_32": dict(cfg=dict(), seed=1, games=4, ticks=1100),
    # combat-heavy: tiny board, NPCs, short episodes
    "small_npc_random": dict(cfg=dict(width=6, height=6, n_npcs=4, max_ticks=60), seed=2,
                             games=24, ticks=260),
    # player deaths (no tick limit) on a 5x5 board
    "duel_5": dict(cfg=dict(width=5, height=5, max_ticks=0), seed=3, games=24, ticks=700),
    # deep multi-depth play, despawn Unreachable
    "stairs_unreachable": dict(cfg=dict(width=8, height=7, max_ticks=150, policy=(2, 2)), seed=4,
                               games=16, ticks=320),
    # despawn Unused: regenerated depths (generation 1)
    "stairs_unused": dict(cfg=dict(width=7, height=8, max_ticks=150, despawn=2, policy=(2, 1)),
                          seed=5, games=16, ticks=320),
    "stairs_unused_both": dict(cfg=dict(width=6, height=6, max_ticks=120, despawn=2,
                                        policy=(2, 2), n_npcs=2), seed=6, games=16, ticks=260),
    # Separated start, both strategies
    "separated_unreachable": dict(cfg=dict(width=6, height=7, max_ticks=120, start_mode=2,
                                           p1_depth=0, p2_depth=3, policy=(2, 1), n_npcs=3),
                                  seed=7, games=12, ticks=260),
    "separated_unused": dict(cfg=dict(width=7, height=6, max_ticks=120, start_mode=2, despawn=2,
                                      p1_depth=2, p2_depth=0, policy=(1, 2)), seed=8, games=12,
                             ticks=260),
    # Unused despawn, Separated start: player 1 leaves the NPCs' depth, which
    # is despawned; player 2 descends into its regeneration, whose staircase
    # can lie under an NPC -- handle_move attacks it (pos_lookup before the
    # tile, updater.py:199-207); 21 such attacks in these games
    "npc_stair_unused_sep": dict(cfg=dict(width=6, height=6, max_ticks=200, start_mode=2,
                                          despawn=2, p1_depth=1, p2_depth=0, n_npcs=10,
                                          policy=(2, 2)), seed=15, games=16, ticks=300),
    # C3 shape: 64x64, K=8 NPCs, random
    "c3_npc_64": dict(cfg=dict(width=64, height=64, n_npcs=8), seed=3, games=6, ticks=300),
    # C3 at full episode length: 64x64, K=8, max_ticks 1000, past the first
    # autoreset (NPC hits and kills, descents, episode ends)
    "c3_npc_64_long": dict(cfg=dict(width=64, height=64, n_npcs=8), seed=31, games=32,
                           ticks=1100),
    # C5 shape: 128x128, both StaircaseBot ("ladder"), Unreachable, past the
    # first autoreset
    "c5_stairs_128": dict(cfg=dict(width=128, height=128, policy=(2, 2)), seed=51, games=12,
                          ticks=1100),
    # minimum board (W=H=4: staircase fixed at (1,1), no dungeon draws)
    "tiny_4": dict(cfg=dict(width=4, height=4, max_ticks=40, n_npcs=1, policy=(1, 2)), seed=9,
                   games=16, ticks=200),
    # non-square, game_offset != 0, seed > 2^32
    "offset_seed": dict(cfg=dict(width=9, height=5, max_ticks=80, n_npcs=2), seed=(7 << 32) | 11,
                        games=8, ticks=200, offset=1000),
    # explicit-grid dungeon bank: interior walls, open borders, NPCs, random play
    "bank_random_npc": dict(cfg=dict(width=9, height=8, max_ticks=90, n_npcs=3,
                                     layouts=make_layouts(9, 8, 4, 101, open_border=True)),
                            seed=12, games=16, ticks=300),
    # bank + StaircaseBot deep play under Unused (regenerated layouts), 2-3 staircases
    "bank_stairs_unused": dict(cfg=dict(width=8, height=9, max_ticks=150, despawn=2,
                                        policy=(2, 1), n_npcs=2,
                                        layouts=make_layouts(8, 9, 3, 102, n_stairs=(1, 3, 2))),
                               seed=13, games=16, ticks=320),
    # stock-seed mode: the unmodified reference with random.seed(n) / np.random.seed(n)
    "stock_c1_random": dict(cfg=dict(rng=1), seed=1000, games=4, ticks=1100),
    "stock_npc_stairs": dict(cfg=dict(rng=1, width=7, height=8, max_ticks=150, n_npcs=3,
                                      policy=(2, 1)), seed=2000, games=16, ticks=320),
    "stock_unused_separated": dict(cfg=dict(rng=1, width=6, height=6, max_ticks=120, despawn=2,
                                            start_mode=2, p1_depth=0, p2_depth=2, n_npcs=2,
                                            policy=(1, 2)), seed=3000, games=16, ticks=260),
    "stock_bank_unreachable": dict(cfg=dict(rng=1, width=8, height=9, max_ticks=150,
                                            policy=(2, 2), n_npcs=2,
                                            layouts=make_layouts(8, 9, 3, 104, n_stairs=(1, 2))),
                                   seed=4000, games=12, ticks=320),
    # stock-seed mode with a depth gap beyond 256 (player 2 starts 260 levels
    # down): player 1's StaircaseBot creates depths 1..259, then enters the
    # depths player 2's RandomBot created and left -- each a dungeon the
    # engine must recall from player 2's dstore ring (the former depth-mod-256
    # store had overwritten them with player 1's shallow depths)
    "stock_deep_gap": dict(cfg=dict(rng=1, width=5, height=5, max_ticks=1500, start_mode=2,
                                    p1_depth=0, p2_depth=260, policy=(2, 1)), seed=5000, games=4,
                           ticks=1100),
    # a one-layout bank (no dungeon draw), Separated start, both StaircaseBots
    # dense NPCs (more than the engine's 16 register slots: its occupancy-grid
    # form); the reference's updater takes any number of entities
    "dense_npc_12x12": dict(cfg=dict(width=12, height=12, n_npcs=30, npc_health=2,
                                     max_ticks=120), seed=61, games=12, ticks=300),
    "dense_npc_64": dict(cfg=dict(width=64, height=64, n_npcs=32), seed=62, games=8, ticks=400),
    "dense_npc_stairs": dict(cfg=dict(width=10, height=9, n_npcs=20, max_ticks=100, despawn=2,
                                      policy=(2, 1)), seed=63, games=12, ticks=260),
    # games whose first tick's draws overflow the tick block (fallback streams)
    "overflow_shuffle": dict(cfg=dict(width=6, height=6, max_ticks=30), seed=5, games=3,
                             ticks=40, offset=("shuffle", 5, 0, 1)),
    "overflow_policy": dict(cfg=dict(width=6, height=6, max_ticks=30), seed=5, games=3,
                            ticks=40, offset=("policy", 5, 0, 1)),
    "bank_single_separated": dict(cfg=dict(width=7, height=7, max_ticks=100, start_mode=2,
                                           p1_depth=1, p2_depth=0, policy=(2, 2),
                                           layouts=make_layouts(7, 7, 1, 103, n_stairs=(2,))),
                                  seed=14, games=12, ticks=260),
}


# moving NPCs (npc_policy: 1 RANDOM, 2 CHASE; NpcAiUpdater): the reference's
# own NPC shuffle, NPC-vs-player and NPC-vs-NPC combat (Block / Ambush / Flee),
# a player's hit on an NPC that moves (Flee), NPC deaths on a staircase
# (updater.py:263-270), all on register (<= 16) and dense NPC forms
CASES.update({
    "mnpc_random_12x12": dict(cfg=dict(width=12, height=12, n_npcs=24, npc_health=2,
                                       max_ticks=120, npc_policy=1), seed=71, games=12,
                              ticks=300),
    "mnpc_c3_64": dict(cfg=dict(width=64, height=64, n_npcs=8, npc_policy=1), seed=72, games=8,
                       ticks=400),
    "mnpc_stairs_unused": dict(cfg=dict(width=10, height=9, n_npcs=12, max_ticks=100, despawn=2,
                                        policy=(2, 2), npc_policy=1), seed=73, games=12,
                               ticks=300),
    "mnpc_stairs_dense": dict(cfg=dict(width=11, height=10, n_npcs=28, npc_health=2,
                                       max_ticks=100, policy=(2, 1), npc_policy=1), seed=74,
                              games=12, ticks=300),
    "mnpc_chase_8x8": dict(cfg=dict(width=8, height=8, n_npcs=6, npc_damage=2, max_ticks=60,
                                    npc_policy=2), seed=75, games=16, ticks=260),
    "mnpc_chase_dense": dict(cfg=dict(width=16, height=14, n_npcs=40, npc_health=2,
                                      max_ticks=150, policy=(2, 1), npc_policy=2), seed=76,
                             games=10, ticks=320),
    "mnpc_separated": dict(cfg=dict(width=7, height=7, max_ticks=150, start_mode=2, p1_depth=3,
                                    p2_depth=0, n_npcs=6, policy=(2, 2), npc_policy=1), seed=77,
                           games=12, ticks=300),
    "mnpc_bank": dict(cfg=dict(width=9, height=8, max_ticks=90, n_npcs=6, npc_policy=1,
                               layouts=make_layouts(9, 8, 4, 105, open_border=True)),
                      seed=78, games=12, ticks=260),
    "mnpc_stock": dict(cfg=dict(rng=1, width=8, height=8, n_npcs=6, max_ticks=80, policy=(1, 2),
                                npc_policy=1), seed=7000, games=12, ticks=240),
})


def sweep_case(case, base=1000):
    """Draw `case` of tests/test_gpu_fuzz.py's random-configuration sweep as a
    fixture spec (reference semantics only: the players' 10 / 2 / 1, up to 6
    games) -- the same configuration the GPU sweep runs engine vs oracle."""
    sys.path.insert(0, os.path.dirname(HERE))
    from test_gpu_fuzz import _draw
    cfg, layouts, B, T, seed, off, pol, _ = _draw(case, base)
    assert not cfg["flags"] and 3 not in pol, "not a reference-semantics draw"
    cfg = dict(cfg, player_health=10, player_damage=2, player_armor=1, policy=pol,
               layouts=layouts)
    return dict(cfg=cfg, seed=seed, games=min(B, 6), ticks=T, offset=off)


# random-configuration sweep draws with the most going on (tests/golden/
# sweep_reference.py checks every such draw; these are kept as fixtures so
# the GPU golden tests -- step, events, rollout, codec -- run on them too)
CASES.update({
    "sweep_94_sep_unused": sweep_case(94),          # 4x27, 158 descents
    "sweep_151_bank_stock": sweep_case(151),        # 13x6 bank, stock seeding, 302 combats
    "sweep_174_bank_dense": sweep_case(174),        # 21x24 bank, 106 NPCs, Separated
    "sweep_196_dense_stock": sweep_case(196),       # 39x33, 227 NPCs, stock, Separated
})

SNAP_KEYS_I32 = ["p_x", "p_y", "p_depth", "p_health", "st_x", "st_y", "tick", "status",
                 "episode", "ret_sum", "ep_count", "counters", "npc_pos", "npc_health",
                 "npc_alive"]


def run_case(R, name, spec):
    cfg = dict(DEFAULT_CFG)
    cfg.update(spec["cfg"])
    seed, G, T = spec["seed"], spec["games"], spec["ticks"]
    off = spec.get("offset", 0)
    if isinstance(off, tuple):   # (kind, seed, episode, tick): search the game id
        kind, s_, e_, t_ = off
        off = find_reservoir_overflow(s_, e_, t_, kind)
        print(f"{name}: game {off} overflows the {kind} reservoir at tick {t_}")
    hs = [Harness(R, cfg, seed, off + g) for g in range(G)]
    bank = cfg.get("layouts")
    keys = SNAP_KEYS_I32 + (["p_layout"] if bank is not None else [])
    snaps = {k: [] for k in keys}
    actions = np.zeros((T, G, 2), np.int8)
    world_len = np.zeros((T + 1, G), np.int32)
    world = []
    ev_len = np.zeros((T, G), np.int32)
    events = []
    ent_len = np.zeros((T + 1, G), np.int32)
    ents = []

    def record(t):
        recs = [h.snapshot() for h in hs]
        for k in keys:
            snaps[k].append([r[k] for r in recs])
        for g, r in enumerate(recs):
            world_len[t, g] = len(r["world"])
            world.extend(r["world"])
            ent_len[t, g] = len(r["entities"])
            ents.extend(r["entities"])

    import optimax_rogue.networking.serializer as ser
    ser_ticks = sorted(set([0, T // 4, T // 2, (3 * T) // 4, T]))
    ser_blobs, ser_len = [], np.zeros((len(ser_ticks), G), np.int32)

    def record_ser(t):
        if t in ser_ticks:
            j = ser_ticks.index(t)
            for g, h in enumerate(hs):
                b = ser.serialize(h.gs)
                ser_len[j, g] = len(b)
                ser_blobs.append(b)

    record(0)
    record_ser(0)
    for t in range(T):
        for g, h in enumerate(hs):
            a = h.policy()
            actions[t, g] = a
            evs = h.step(a)
            ev_len[t, g] = len(evs)
            events.extend(evs)
        record(t + 1)
        record_ser(t + 1)

    cfg_js = {k: v for k, v in cfg.items() if k != "layouts"}
    cfg_js["n_layouts"] = 0 if bank is None else int(len(bank))
    out = {"cfg_json": np.frombuffer(json.dumps(cfg_js).encode(), np.uint8),
           "seed": np.array([seed], np.uint64), "game_offset": np.array([off], np.int64),
           "actions": actions, "world_len": world_len,
           "world": np.array(world, np.int32).reshape(-1, 3 if bank is None else 4),
           "event_len": ev_len, "events": np.array(events, np.int32).reshape(-1, 4),
           "entity_len": ent_len, "entities": np.array(ents, np.int32).reshape(-1, 5),
           "ser_ticks": np.array(ser_ticks, np.int32), "ser_len": ser_len,
           "ser_bytes": np.frombuffer(b"".join(ser_blobs), np.uint8)}
    if bank is not None:
        out["layouts"] = np.ascontiguousarray(bank, np.uint8)
    for k in keys:
        a = np.array(snaps[k])
        if a.ndim == 3:  # [T+1, G, F] -> [T+1, F, G] (engine SoA layout)
            a = a.transpose(0, 2, 1)
        dt = {"npc_pos": np.uint16, "npc_health": np.int8, "npc_alive": np.uint32,
              "p_layout": np.int16}.get(k, np.int32)
        out[k] = np.ascontiguousarray(a.astype(dt))
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    st = out["status"][1:]
    print(f"{name}: {G} games x {T} ticks, finished episodes={int(out['ep_count'][-1].sum())}, "
          f"combats={int(out['counters'][-1][0].sum())}, descents={int(out['counters'][-1][1].sum())}, "
          f"dungeons={int(out['counters'][-1][2].sum())}, npc deaths={int(out['counters'][-1][3].sum())}, "
          f"max depth={int(out['p_depth'].max())}, statuses={sorted(set(st.ravel().tolist()))}, "
          f"bytes={os.path.getsize(path)}")
    if cfg.get("npc_policy"):   # what the moving NPCs did (event records)
        ev = out["events"]
        tally = {}
        for t_, i_, a_, b_ in ev.tolist():
            who = "npc" if i_ >= 3 else "player"
            if t_ == 1:
                k = f"{who}->{'npc' if a_ >= 3 else 'player'}:{['', 'Block', 'Ambush', 'Flee', 'Parry'][b_]}"
            elif t_ == 3:
                k = f"{who} move"
            elif t_ == 2:
                k = "npc death"
            else:
                k = f"type{t_}"
            tally[k] = tally.get(k, 0) + 1
        print("   ", dict(sorted(tally.items())))


# --------------------------------------------------------------------------
# Known-answer scenarios (SURVEY.md s4's semantics probes): hand-built states
# on an 8x8 board (staircase at (5, 5); players health 10, damage 2, armor 1)
# stepped once by the reference updater, initiative chosen by the seed
# --------------------------------------------------------------------------
KAT_CFG = dict(DEFAULT_CFG, width=8, height=8, n_npcs=2, npc_health=3, npc_damage=1,
               npc_armor=0, max_ticks=1000)
# name: (p1 (x, y, hp), p2 (x, y, hp), NPCs [(x, y, hp)], (m1, m2), p1 first)
KAT_SCENARIOS = {
    "swap_p1_first": ((2, 2, 10), (3, 2, 10), [], (2, 4), True),
    "swap_p2_first": ((2, 2, 10), (3, 2, 10), [], (2, 4), False),
    "block": ((2, 2, 10), (3, 2, 10), [], (2, 5), True),
    "same_target_p1_first": ((2, 2, 10), (4, 2, 10), [], (2, 4), True),
    "same_target_p2_first": ((2, 2, 10), (4, 2, 10), [], (2, 4), False),
    "chase_p1_first": ((2, 2, 10), (3, 2, 10), [], (2, 2), True),
    "chase_p2_first": ((2, 2, 10), (3, 2, 10), [], (2, 2), False),
    "wall": ((1, 3, 10), (4, 4, 10), [], (4, 5), True),
    "descend": ((4, 5, 10), (2, 2, 10), [], (2, 5), True),
    "both_descend_p1_first": ((4, 5, 10), (5, 4, 10), [], (2, 3), True),
    "both_descend_p2_first": ((4, 5, 10), (5, 4, 10), [], (2, 3), False),
    "npc_kill": ((2, 4, 10), (6, 6, 10), [(3, 4, 1)], (2, 5), True),
    "npc_both_hit": ((2, 3, 10), (4, 3, 10), [(3, 3, 2), (6, 6, 3)], (2, 4), False),
    "mutual_kill": ((2, 2, 1), (3, 2, 1), [], (2, 4), True),
    "kill_then_step": ((2, 2, 10), (3, 2, 1), [], (2, 1), True),
    # an NPC standing on the staircase (possible after an Unused despawn
    # regenerates its depth): stepping onto it is a combat, not a descent
    "npc_on_stairs": ((4, 5, 10), (2, 2, 10), [(5, 5, 3)], (2, 5), True),
}


def kat_seed(p1_first):
    """Smallest seed whose tick block (game 0, episode 0, tick 1) lets player
    1 act first (CPython shuffle of [p1, p2]: randbelow(2) == 1) or not."""
    for seed in range(1 << 20):
        tb = TickBits(seed, 0, 0, 1, PUR_SHUFFLE)
        r = tb.getrandbits(2)
        while r >= 2:
            r = tb.getrandbits(2)
        if (r == 1) == p1_first:
            return seed
    raise RuntimeError("no seed")


def make_scenarios(R):
    names = list(KAT_SCENARIOS)
    n = len(names)
    init = np.zeros((n, 4, 5), np.int32)       # entities {iden, depth, x, y, health}, -1 = none
    init[:, :, 0] = -1
    moves = np.zeros((n, 2), np.int8)
    seeds = np.zeros(n, np.uint64)
    ev_len = np.zeros(n, np.int32)
    events = []
    final = {k: [] for k in ("p_x", "p_y", "p_depth", "p_health", "st_x", "st_y", "tick",
                             "status", "npc_health", "npc_alive")}
    ent_len = np.zeros(n, np.int32)
    ents = []
    for i, name in enumerate(names):
        (x1, y1, h1), (x2, y2, h2), npcs, (m1, m2), first = KAT_SCENARIOS[name]
        seed = kat_seed(first)
        h = Harness(R, KAT_CFG, seed, 0)
        tiles = np.full((8, 8), int(R.world.Tile.Ground), np.int32)
        tiles[[0, -1], :] = int(R.world.Tile.Wall)
        tiles[:, [0, -1]] = int(R.world.Tile.Wall)
        tiles[5, 5] = int(R.world.Tile.StaircaseDown)
        Ent = R.entities.Entity
        es = [Ent(1, 0, x1, y1, h1, 10, 2, 1, [], dict()), Ent(2, 0, x2, y2, h2, 10, 2, 1, [], dict())]
        for k, (nx, ny, nh) in enumerate(npcs):
            es.append(Ent(3 + k, 0, nx, ny, nh, 3, 1, 0, [], dict()))
        h.gs = R.state.GameState(True, 1, 1, 2, R.world.World({0: R.world.Dungeon(tiles)}), es)
        h.gens = {0: 1}
        for j, e in enumerate(es):
            init[i, j] = (e.iden, e.depth, e.x, e.y, e.health)
        moves[i] = (m1, m2)
        seeds[i] = seed
        evs = h.step([m1, m2])
        ev_len[i] = len(evs)
        events.extend(evs)
        snap = h.snapshot()
        for k in final:
            final[k].append(snap[k])
        ent_len[i] = len(snap["entities"])
        ents.extend(snap["entities"])
        print(f"kat {name}: seed {seed}, events {evs}, status {snap['status']}")
    out = dict(names=np.array(names), init=init, moves=moves, seeds=seeds, ev_len=ev_len,
               events=np.array(events, np.int32).reshape(-1, 4), ent_len=ent_len,
               ents=np.array(ents, np.int32).reshape(-1, 5),
               cfg_json=np.frombuffer(json.dumps(KAT_CFG).encode(), np.uint8))
    for k, v in final.items():
        out["final_" + k] = np.array(v, np.int64)
    np.savez_compressed(os.path.join(HERE, "kat_scenarios.npz"), **out)


def philox_kat():
    """Random123 known-answer vectors for Philox4x32-10 (kat_vectors)."""
    return [
        ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
        ((M, M, M, M), (M, M), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
        ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
         (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
    ]


def main():
    for ctr, key, want in philox_kat():
        assert philox4x32_10(ctr, key) == want
    R = import_reference()
    only = sys.argv[1:]
    if not only or "kat" in only:
        make_scenarios(R)
    for name, spec in CASES.items():
        if only and name not in only:
            continue
        run_case(R, name, spec)


if __name__ == "__main__":
    main()
