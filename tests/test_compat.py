"""CPU: the reference-schema views (compat.game_state) drive the reference's
own bots unchanged.  The snapshots come from the oracle; the bots are the
reference's RandomBot / StaircaseBot classes when /root/reference is present
in this (build) container, otherwise the test is skipped."""
import os
import sys

import numpy as np
import pytest

from optimax_rogue_amd import EnvConfig, Move
from optimax_rogue_amd.compat import game_state

REF = "/root/reference"


def _ref_bots():
    if not os.path.isdir(REF):
        pytest.skip("reference not present (GPU box)")
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_golden  # installs the inflection stub + import path only
    R = make_golden.import_reference()
    return R


def test_views_schema(oracle_lib):
    cfg = EnvConfig(width=9, height=8, n_npcs=3, max_ticks=100)
    o = oracle_lib.Oracle(cfg.to_dict(), 16, 4)
    o.reset()
    o.rollout(2, 1, 40)
    snap = o.export()
    for i in range(16):
        gs = game_state(snap, i, cfg)
        ents = o.entities(i)
        assert sorted((e.iden, e.depth, e.x, e.y, e.health) for e in gs.entities) == \
            sorted(e[:5] for e in ents)
        for p in (1, 2):
            me = gs.iden_lookup[p]
            d = gs.world.dungeons[me.depth]
            assert d.tiles.shape == (9, 8)
            assert (d.tiles == 2).sum() == 2 * 9 + 2 * 8 - 4
            assert d.staircase() == (snap["st_x"][p - 1][i], snap["st_y"][p - 1][i])
            assert gs.pos_lookup[(me.depth, me.x, me.y)] is me
            v = gs.view_for(me)
            assert list(v.world.dungeons) == [me.depth]
            assert all(e.depth == me.depth for e in v.entities)
        world = dict((w[0], (w[1], w[2])) for w in o.world(i))
        for depth, dv in gs.world.dungeons.items():
            assert world[depth] == dv.staircase()


def test_reference_staircasebot_on_views(oracle_lib):
    R = _ref_bots()
    cfg = EnvConfig(width=10, height=7, max_ticks=80)
    B = 32
    o = oracle_lib.Oracle(cfg.to_dict(), B, 9)
    o.reset()
    bots = [[R.staircasebot.StaircaseBot(1 + p) for _ in range(B)] for p in range(2)]
    for t in range(60):
        snap = o.export()
        want = o.policy(2, 2)
        got = np.zeros_like(want)
        for i in range(B):
            gs = game_state(snap, i, cfg)
            for p in range(2):
                got[i, p] = int(bots[p][i].move(gs.view_for(gs.iden_lookup[1 + p])))
        assert np.array_equal(got, want), t
        o.step(want)


def test_reference_randombot_on_views(oracle_lib):
    R = _ref_bots()
    cfg = EnvConfig(width=8, height=8)
    o = oracle_lib.Oracle(cfg.to_dict(), 4, 1)
    o.reset()
    snap = o.export()
    bot = R.randombot.RandomBot(1)
    import random as _r
    R.randombot.random = _r.Random(0)   # the module's own RNG, as in the stock bot runner
    for i in range(4):
        gs = game_state(snap, i, cfg)
        assert Move(int(bot.move(gs.view_for(gs.iden_lookup[1])))) in list(Move)


def oracle_view(o, g, cfg):
    """GameStateView from the oracle's own world dict (exact insertion order)
    and entity list."""
    from optimax_rogue_amd.compat import DungeonView, EntityView, GameStateView, WorldView
    dungeons = {}
    for w in o.world(g):   # (depth, sx, sy[, bank layout])
        tiles = o.layouts[w[3]] if len(w) > 3 else None
        dungeons[w[0]] = DungeonView(cfg.width, cfg.height, w[1], w[2], tiles=tiles)
    ents = []
    for iden, depth, x, y, hp, dmg, arm in o.entities(g):
        base = cfg.player_health if iden <= 2 else cfg.npc_health
        ents.append(EntityView(iden, depth, x, y, hp, base, dmg, arm))
    return GameStateView(True, int(o.export()["tick"][g]), WorldView(dungeons), ents)


@pytest.mark.parametrize("name", __import__("golden_util").case_names())
def test_wire_codec_matches_reference_bytes(oracle_lib, name):
    """GameState -> serializer.serialize bytes (JSON envelope, a85 body, world
    and entity encodings) equal the reference's bytes at the sampled ticks."""
    from golden_util import Fixture
    fx = Fixture(name)
    cfg = EnvConfig.from_dict(fx.cfg, layouts=fx.layouts)
    o = oracle_lib.Oracle(fx.cfg, fx.G, fx.seed, fx.game_offset, layouts=fx.layouts)
    o.reset(episode=np.zeros(fx.G, np.int32))
    ticks = set(int(t) for t in fx.z["ser_ticks"])
    for t in range(fx.T + 1):
        if t in ticks:
            for g in range(fx.G):
                assert oracle_view(o, g, cfg).serialize() == fx.serialized(t, g), (name, t, g)
        if t < fx.T:
            o.step(o.policy(*fx.policy))


def test_world_depths_rule(oracle_lib):
    """compat.world_depths (the derived World.dungeons set) equals the oracle's
    explicit dict for every fixture tick (order too, for Together starts)."""
    from golden_util import Fixture, case_names
    from optimax_rogue_amd.compat import world_depths
    for name in case_names():
        fx = Fixture(name)
        cfg = EnvConfig.from_dict(fx.cfg)
        for t in range(0, fx.T + 1, 7):
            s = fx.state(t)
            for g in range(fx.G):
                want = [w[0] for w in fx.world(t, g)]
                got = world_depths(cfg, int(s["p_depth"][0][g]), int(s["p_depth"][1][g]))
                if cfg.start_mode == 1 and cfg.despawn == 1:
                    assert got == want, (name, t, g)
                else:
                    assert sorted(got) == sorted(want), (name, t, g)


def test_dungeon_bank_tables():
    """DungeonBank's precomputed tables equal the reference Dungeon methods'
    results: Ground list = get_random_unblocked's candidates (x-major flat
    order, world.py:57-66), staircase = first StaircaseDown (world.py:52-55)."""
    from golden_util import Fixture
    from optimax_rogue_amd import DungeonBank
    fx = Fixture("bank_stairs_unused")
    bank = DungeonBank(fx.layouts)
    L, W, H = fx.layouts.shape
    for li in range(L):
        t = fx.layouts[li].astype(np.int32)
        avail = t == 1
        want = np.arange(W * H).reshape(W, H)[avail]
        n = int(bank.meta[li, 0])
        assert n == len(want) and np.array_equal(bank.ground[li, :n], want)
        assert bank.staircase(li) == tuple(int(v) for v in np.argwhere(t == 3)[0])
    with pytest.raises(ValueError):
        DungeonBank(np.ones((1, 5, 5), np.uint8))          # no staircase
    with pytest.raises(ValueError):
        DungeonBank(np.full((1, 5, 5), 7, np.uint8))       # not a Tile code


def test_reference_staircasebot_on_bank_views(oracle_lib):
    """The reference's StaircaseBot on views of an explicit-grid game walks
    to the bank layout's first staircase, as the oracle's policy does."""
    R = _ref_bots()
    from golden_util import Fixture
    fx = Fixture("bank_single_separated")
    from optimax_rogue_amd import DungeonBank
    bank = DungeonBank(fx.layouts)
    cfg = EnvConfig.from_dict(fx.cfg, layouts=fx.layouts)
    B = fx.G
    o = oracle_lib.Oracle(fx.cfg, B, fx.seed, 0, layouts=fx.layouts)
    o.reset()
    bots = [[R.staircasebot.StaircaseBot(1 + p) for _ in range(B)] for p in range(2)]
    for t in range(40):
        snap = o.export()
        want = o.policy(2, 2)
        got = np.zeros_like(want)
        for i in range(B):
            gs = game_state(snap, i, cfg, bank=bank)
            for p in range(2):
                got[i, p] = int(bots[p][i].move(gs.view_for(gs.iden_lookup[1 + p])))
        assert np.array_equal(got, want), t
        o.step(want)
