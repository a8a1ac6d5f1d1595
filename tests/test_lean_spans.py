"""The paired StaircaseBot form's lean spans (pair_rollout_kernel, kLean;
built with -DORX_LEAN=1 -- `python -m optimax_rogue_amd.build --variant lean`
-- and off by default: measured slower), checked on the CPU
against the oracle: the span the kernel computes after a
general tick -- min(distance to the staircase - 1 over both players, (the
players' distance - 1) / 2 on one depth, ticks before the episode limit; 0
for a finished game or, with separation damage across depths, when the next
tick's damage would kill) -- must only cover ticks that are plain greedy
walks (reference: optimax_rogue_bots/staircasebot.py:9-21 for the move,
optimax_rogue/logic/updater.py:76-162 for the tick) plus the separation
damage the lean tick applies, and a span decremented by one tick must stay
covered by the span recomputed from the next state (the kernel decrements,
it does not recompute, inside a lean run).  No GPU: the oracle is the ground
truth; the separation timer is tracked here as the kernel keeps it."""
import numpy as np
import pytest

from optimax_rogue_amd.enums import Move

IN_PROGRESS = 1


def sep_damage(ex, sep, period):
    """The next tick's separation damage per player [2, B] (0 on one depth):
    ceil(k / period), k = t0 - start + 1, the shallower player only."""
    d, t0 = ex["p_depth"], ex["tick"]
    k = t0 - np.where(sep < 0, t0, sep) + 1
    dmg = (k + period - 1) // period
    differ = d[0] != d[1]
    return np.stack([np.where(differ & (d[0] < d[1]), dmg, 0),
                     np.where(differ & (d[1] < d[0]), dmg, 0)])


def lean_span(ex, max_ticks, period=0, sep=None):
    """The kernel's span from an exported state (per game); period > 0:
    separation damage on (sep: the games' separation start, -1 unset)."""
    x, y, d = ex["p_x"], ex["p_y"], ex["p_depth"]
    sx, sy = ex["st_x"], ex["st_y"]
    dist = np.abs(sx - x) + np.abs(sy - y)              # [2, B]
    sp = dist.min(axis=0) - 1
    m = np.abs(x[0] - x[1]) + np.abs(y[0] - y[1])
    sp = np.where(d[0] == d[1], np.minimum(sp, (m - 1) >> 1), sp)
    if period:
        dead = (ex["p_health"] - sep_damage(ex, sep, period) <= 0).any(axis=0)
        sp = np.where(dead, 0, sp)
    if max_ticks:
        sp = np.minimum(sp, max_ticks - ex["tick"] - 1)
    return np.where(ex["status"] == IN_PROGRESS, sp, 0)


def track_sep(sep, ex, nxt):
    """The kernel's separation timer after one tick (readme.md:46-47): set at
    the first tick that ends on two depths, cleared on one depth or a reset."""
    running = ex["status"] == IN_PROGRESS
    differ = nxt["p_depth"][0] != nxt["p_depth"][1]
    out = np.where(differ, np.where(sep < 0, ex["tick"], sep), -1)
    return np.where(running, out, -1)


def greedy(ex):
    """StaircaseBot's move and the cell it leads to (both players)."""
    x, y, sx, sy = ex["p_x"], ex["p_y"], ex["st_x"], ex["st_y"]
    dx, dy = sx - x, sy - y
    mv = np.where(np.abs(dx) > np.abs(dy), np.where(dx > 0, int(Move.Right), int(Move.Left)),
                  np.where(dy > 0, int(Move.Down), int(Move.Up)))
    nx = x + (mv == int(Move.Right)) - (mv == int(Move.Left))
    ny = y + (mv == int(Move.Down)) - (mv == int(Move.Up))
    return mv, nx, ny


CASES = {
    "together": dict(width=96, height=96, max_ticks=150),
    "sep_damage": dict(width=96, height=96, max_ticks=120, flags=1, sep_period=4),
    "sep_damage_c5": dict(width=128, height=128, max_ticks=1000, flags=1, sep_period=8),
    "sep_separated_frail": dict(width=40, height=40, start_mode=2, p1_depth=0, p2_depth=2,
                                max_ticks=0, flags=1, sep_period=3, player_health=6),
    "separated": dict(width=80, height=80, start_mode=2, p1_depth=0, p2_depth=1, max_ticks=130),
    "unused_small": dict(width=12, height=10, despawn=2, max_ticks=40),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_lean_spans_cover_plain_ticks(name, oracle_lib):
    cfg = CASES[name]
    B, T = 384, 260
    period = cfg.get("sep_period", 0) if cfg.get("flags", 0) & 1 else 0
    ora = oracle_lib.Oracle(cfg, B, 17, 0)
    ora.reset(episode=np.zeros(B, np.int32))
    ex = ora.export()
    sep = np.full(B, -1, np.int64)
    covered = 0
    for t in range(T):
        span = lean_span(ex, cfg.get("max_ticks", 0), period, sep)
        mv, nx, ny = greedy(ex)
        hp = ex["p_health"] - (sep_damage(ex, sep, period) if period else 0)
        a = ora.policy(2, 2)
        ora.step(a)
        nxt = ora.export()
        on = span > 0
        covered += int(on.sum())
        # a covered tick is a plain greedy walk: the bots' moves, one step
        # each, nothing else of the game changes but its tick
        assert np.array_equal(a.T[:, on], mv[:, on]), (name, t)
        assert np.array_equal(nxt["p_x"][:, on], nx[:, on]), (name, t)
        assert np.array_equal(nxt["p_y"][:, on], ny[:, on]), (name, t)
        for k in ("p_depth", "st_x", "st_y"):
            assert np.array_equal(nxt[k][:, on], ex[k][:, on]), (name, t, k)
        assert np.array_equal(nxt["p_health"][:, on], hp[:, on]), (name, t)
        assert np.array_equal(nxt["tick"][on], ex["tick"][on] + 1), (name, t)
        assert (nxt["status"][on] == IN_PROGRESS).all(), (name, t)
        assert np.array_equal(nxt["episode"][on], ex["episode"][on]), (name, t)
        # the kernel's decremented span (zeroed in the lean tick when the
        # next tick's separation damage kills) stays within the recomputed one
        sep = track_sep(sep, ex, nxt)
        nspan = lean_span(nxt, cfg.get("max_ticks", 0), period, sep)
        carried = span - 1
        if period:
            kills = (nxt["p_health"] - sep_damage(nxt, sep, period) <= 0).any(axis=0)
            carried = np.where(kills, 0, carried)
        assert (nspan[on] >= carried[on]).all(), (name, t)
        ex = nxt
    assert covered > B * T // 10, (name, covered)   # the spans are not vacuous
