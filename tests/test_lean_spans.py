"""The paired StaircaseBot form's lean spans (pair_rollout_kernel, kLean),
checked on the CPU against the oracle: the span the kernel computes after a
general tick -- min(distance to the staircase - 1 over both players, (the
players' distance - 1) / 2 on one depth, ticks before the episode limit; 0
with separation damage across depths or a finished game) -- must only cover
ticks that are plain greedy walks (reference: optimax_rogue_bots/
staircasebot.py:9-21 for the move, optimax_rogue/logic/updater.py:76-162 for
the tick), and a span decremented by one tick must stay covered by the span
recomputed from the next state (the kernel decrements, it does not
recompute, inside a lean run).  No GPU: the oracle is the ground truth."""
import numpy as np
import pytest

from optimax_rogue_amd.enums import Move

IN_PROGRESS = 1


def lean_span(ex, max_ticks, sep):
    """The kernel's span from an exported state (per game)."""
    x, y, d = ex["p_x"], ex["p_y"], ex["p_depth"]
    sx, sy = ex["st_x"], ex["st_y"]
    dist = np.abs(sx - x) + np.abs(sy - y)              # [2, B]
    sp = dist.min(axis=0) - 1
    m = np.abs(x[0] - x[1]) + np.abs(y[0] - y[1])
    same = d[0] == d[1]
    sp = np.where(same, np.minimum(sp, (m - 1) >> 1), 0 if sep else sp)
    if max_ticks:
        sp = np.minimum(sp, max_ticks - ex["tick"] - 1)
    return np.where(ex["status"] == IN_PROGRESS, sp, 0)


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
    "separated": dict(width=80, height=80, start_mode=2, p1_depth=0, p2_depth=1, max_ticks=130),
    "unused_small": dict(width=12, height=10, despawn=2, max_ticks=40),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_lean_spans_cover_plain_ticks(name, oracle_lib):
    cfg = CASES[name]
    B, T = 384, 260
    sep = bool(cfg.get("flags", 0) & 1)
    ora = oracle_lib.Oracle(cfg, B, 17, 0)
    ora.reset(episode=np.zeros(B, np.int32))
    ex = ora.export()
    covered = 0
    for t in range(T):
        span = lean_span(ex, cfg.get("max_ticks", 0), sep)
        mv, nx, ny = greedy(ex)
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
        for k in ("p_depth", "p_health", "st_x", "st_y"):
            assert np.array_equal(nxt[k][:, on], ex[k][:, on]), (name, t, k)
        assert np.array_equal(nxt["tick"][on], ex["tick"][on] + 1), (name, t)
        assert (nxt["status"][on] == IN_PROGRESS).all(), (name, t)
        assert np.array_equal(nxt["episode"][on], ex["episode"][on]), (name, t)
        # the kernel's decremented span stays within the recomputed one
        nspan = lean_span(nxt, cfg.get("max_ticks", 0), sep)
        assert (nspan[on] >= span[on] - 1).all(), (name, t)
        ex = nxt
    assert covered > B * T // 10, (name, covered)   # the spans are not vacuous
