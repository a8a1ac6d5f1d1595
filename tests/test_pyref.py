"""CPU: the pure-Python object-model restatement (oracle/pyref.py, the CPU
baseline's cost model of the reference) against the reference's golden
fixtures -- every tick's SoA state, World.dungeons, update events and
GameState.entities order, for every fixture (all are reference semantics)."""
import numpy as np
import pytest

from golden_util import Fixture, case_names, compare_state


@pytest.mark.parametrize("name", case_names())
def test_pyref_vs_reference_fixture(name):
    from oracle.pyref import Game, batch_state
    fx = Fixture(name)
    cfg = dict(fx.cfg, policy=fx.policy)
    games = [Game(cfg, fx.seed, fx.game_offset + g, layouts=fx.layouts) for g in range(fx.G)]
    compare_state(batch_state(games), fx.state(0), fx.K, f"{name} t=0")
    # the largest fixtures: the whole state every 7th tick (events, world and
    # entity order every tick)
    every = 7 if fx.T * fx.G > 20000 else 1
    for t in range(fx.T):
        for g, game in enumerate(games):
            a = game.policy()
            assert list(fx.actions[t, g]) == a, f"{name} policy t={t} g={g}"
            ev = game.step(*a)
            assert ev == fx.events(t, g), (name, t, g)
            assert game.world_list() == fx.world(t + 1, g), (name, t, g)
            assert game.entity_list() == fx.entities(t + 1, g), (name, t, g)
        if t % every == every - 1 or t == fx.T - 1:
            compare_state(batch_state(games), fx.state(t + 1), fx.K, f"{name} t={t + 1}")


def test_pyref_refuses_extensions():
    from oracle.pyref import Game
    with pytest.raises(ValueError):
        Game(dict(width=8, height=8, flags=1, max_ticks=10, start_mode=1, n_npcs=0), 1, 0)
