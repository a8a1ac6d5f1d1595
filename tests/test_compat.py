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
