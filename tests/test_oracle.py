"""CPU: the C oracle against the reference's golden fixtures (bit-exact), the
Philox known-answer vectors, and the oracle's own invariants."""
import numpy as np
import pytest

from golden_util import Fixture, case_names, compare_state

PHILOX_KAT = [  # Random123 kat_vectors, philox4x32-10
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", PHILOX_KAT)
def test_philox_kat(oracle_lib, ctr, key, want):
    assert oracle_lib.philox(ctr, key) == want


@pytest.mark.parametrize("name", case_names())
def test_oracle_vs_reference_fixture(oracle_lib, name):
    """Every tick: SoA state, World.dungeons dict, update events (type and
    order) and GameState.entities order match the reference."""
    fx = Fixture(name)
    o = oracle_lib.Oracle(fx.cfg, fx.G, fx.seed, fx.game_offset, record_events=True,
                          layouts=fx.layouts)
    o.reset(episode=np.zeros(fx.G, np.int32))
    compare_state(o.export(), fx.state(0), fx.K, f"{name} t=0")
    if fx.layouts is not None:
        assert "p_layout" in o.export()
    for t in range(fx.T):
        a = o.policy(*fx.policy)
        assert np.array_equal(a, fx.actions[t]), f"{name} policy t={t}"
        o.step(a)
        compare_state(o.export(), fx.state(t + 1), fx.K, f"{name} t={t + 1}")
        for g in range(fx.G):
            assert o.world(g) == fx.world(t + 1, g), (name, t, g)
            assert o.events(g) == fx.events(t, g), (name, t, g)
            assert [e[:5] for e in o.entities(g)] == fx.entities(t + 1, g), (name, t, g)


def test_fixtures_cover_the_paths():
    """The committed fixtures exercise every branch the parity claim covers."""
    statuses, flags, events = set(), set(), set()
    despawn, starts, npcs, unused_regen = set(), set(), False, False
    for name in case_names():
        fx = Fixture(name)
        statuses |= set(np.unique(fx.z["status"]).tolist())
        ev = fx.z["events"]
        events |= set(ev[:, 0].tolist())
        flags |= set(ev[ev[:, 0] == 1][:, 3].tolist())
        despawn.add(fx.cfg["despawn"])
        starts.add(fx.cfg["start_mode"])
        npcs |= fx.K > 0 and fx.z["counters"][-1][3].sum() > 0
        if fx.cfg["despawn"] == 2:
            # a dungeon was created on a depth the other player had already left
            unused_regen |= fx.z["counters"][-1][2].sum() > fx.z["counters"][-1][1].sum() * 0.5
    assert {1, 3, 4} <= statuses            # in progress, a win, ties
    assert {1, 2, 3, 4} <= events            # combat, death, position, dungeon created
    assert {1, 2, 3} <= flags                # Block, Ambush, Flee (Parry is dead code)
    assert despawn == {1, 2} and starts == {1, 2}
    assert npcs and unused_regen


def test_oracle_sharding_invariance(oracle_lib):
    cfg = dict(width=9, height=7, n_npcs=3, max_ticks=60)
    full = oracle_lib.Oracle(cfg, 300, 5, 0)
    a = oracle_lib.Oracle(cfg, 100, 5, 0)
    b = oracle_lib.Oracle(cfg, 200, 5, 100)
    for o in (full, a, b):
        o.reset()
        o.rollout(1, 2, 150)
    sf, sa, sb = full.export(), a.export(), b.export()
    for k in sf:
        assert np.array_equal(sf[k], np.concatenate([sa[k], sb[k]], axis=sf[k].ndim - 1)), k


def test_oracle_bad_action_and_freeze(oracle_lib):
    o = oracle_lib.Oracle(dict(width=8, height=8, max_ticks=4, autoreset=0), 4, 1)
    o.reset()
    a = np.full((4, 2), 5, np.int8)
    a[1, 0] = 9
    o.step(a)
    s = o.export()
    assert s["status"].tolist() == [1, 16, 1, 1]
    for _ in range(6):
        o.step(np.full((4, 2), 5, np.int8))
    s = o.export()
    assert s["tick"].tolist() == [4, 1, 4, 4] and s["status"].tolist() == [4, 16, 4, 4]
