"""The readme's character mechanics (readme.md:44, 72, 74): mana -> damage,
heal, experience / leveling, item drops and pickup.  The reference has no
code for them, so nothing the reference outputs can pin them ("parity
unpinned"): the oracle's restatement is checked here against hand-computed
one- and two-tick scenarios (CPU), and the engine against the oracle, bit for
bit, on thousands of games (GPU).  Semantics: include/orx.h ORX_EXT_MANA /
HEAL / LEVELING / ITEMS, DESIGN.md s10."""
import numpy as np
import pytest

MANA, HEAL, LEVEL, ITEMS = 4, 8, 16, 32
STAY, RIGHT, HEAL_MOVE = 5, 2, 6
BASE = dict(width=8, height=8, max_ticks=0, n_npcs=1, npc_health=10, mana_max=9, mana_regen=1,
            mana_per_point=1, xp_per_kill=1, xp_per_level=3, item_drop_pct=100, item_bonus=1,
            item_slots=3)
# player 1 at (2,2) next to the NPC at (3,2); player 2 far away; stairs (6,1)
ENTS = [(1, 0, 2, 2, 10), (2, 0, 5, 5, 10), (3, 0, 3, 2, 10)]


def _one(oracle_lib, flags, ents=ENTS, moves=((RIGHT, STAY),), seed=3, **kw):
    cfg = dict(BASE, flags=flags, **kw)
    o = oracle_lib.Oracle(cfg, 1, seed, 0, record_events=True)
    o.reset(episode=np.zeros(1, np.int32))
    o.set_game(0, ents, (6, 1))
    evs = []
    for m in moves:
        o.step(np.array([m], np.int8))
        evs.append(o.events(0))
    return o.export(), evs


def _rpg(ex, p, field):
    from optimax_rogue_amd.enums import RPG_FIELDS
    return int(ex["p_rpg"][RPG_FIELDS.index(field), p, 0])


def test_mana_attack(oracle_lib):
    """An attack spends up to a third of the bar (9 // 3 = 3) as +3 damage:
    (2 - 1) + 3 = 4 to the NPC; the bar then regenerates 1."""
    ex, evs = _one(oracle_lib, MANA)
    assert int(ex["npc_health"][0, 0]) == 10 - 4
    assert _rpg(ex, 0, "mana") == 9 - 3 + 1
    assert _rpg(ex, 1, "mana") == 9            # capped at the bar
    assert evs[0] == [(1, 1, 3, 1)]             # one Block combat, no other update
    # a low bar: 2 mana give 2 points, mana_per_point 2 -> 1 point for 2 mana
    ex, _ = _one(oracle_lib, MANA, mana_max=6, mana_per_point=2)
    assert int(ex["npc_health"][0, 0]) == 10 - (1 + 1)
    assert _rpg(ex, 0, "mana") == 6 - 2 + 1


def test_no_mana_flag_is_reference_damage(oracle_lib):
    ex, _ = _one(oracle_lib, 0)
    assert int(ex["npc_health"][0, 0]) == 10 - 1
    assert "p_rpg" not in ex


def test_heal(oracle_lib):
    """A heal is a Stay converting up to 3 mana into 3 health, never above the
    max; reported as EntityHealthUpdate(+amount)."""
    hurt = [(1, 0, 2, 2, 5), (2, 0, 5, 5, 9), (3, 0, 3, 2, 10)]
    ex, evs = _one(oracle_lib, MANA | HEAL, ents=hurt, moves=((HEAL_MOVE, HEAL_MOVE),))
    assert ex["p_health"][:, 0].tolist() == [8, 10]
    assert _rpg(ex, 0, "mana") == 9 - 3 + 1
    assert _rpg(ex, 1, "mana") == 9            # spent 1, regained 1
    assert sorted(evs[0]) == [(5, 1, 3, 0), (5, 2, 1, 0)]
    assert ex["p_x"][:, 0].tolist() == [2, 5]   # healing players do not move
    # at full health a heal spends nothing and reports nothing
    ex, evs = _one(oracle_lib, MANA | HEAL, moves=((HEAL_MOVE, STAY),))
    assert _rpg(ex, 0, "mana") == 9 and evs[0] == []
    # the move code is an invalid action without the flag
    ex, _ = _one(oracle_lib, MANA, moves=((HEAL_MOVE, STAY),))
    assert int(ex["status"][0]) == 16


def test_healer_blocks_an_attacker(oracle_lib):
    """A healer counts as staying: player 2 walking into it is Blocked."""
    ents = [(1, 0, 2, 2, 6), (2, 0, 3, 2, 10)]
    ex, evs = _one(oracle_lib, MANA | HEAL, ents=ents, moves=((HEAL_MOVE, 4),), n_npcs=0)
    comb = [e for e in evs[0] if e[0] == 1]
    assert comb == [(1, 2, 1, 1)]              # attacker 2, defender 1, Block
    # damage (2 - 1) + 3 mana; the heal adds 3 before or after it (initiative)
    assert int(ex["p_health"][0, 0]) == 6 + 3 - 4


def test_leveling_refills(oracle_lib):
    """The killing blow's player gains xp_per_kill; crossing a level refills
    health and mana."""
    ents = [(1, 0, 2, 2, 4), (2, 0, 5, 5, 10), (3, 0, 3, 2, 1)]
    ex, evs = _one(oracle_lib, MANA | LEVEL, ents=ents, xp_per_level=1)
    assert (2, 3, 0, 0) in evs[0]               # the NPC died
    assert _rpg(ex, 0, "xp") == 1 and _rpg(ex, 1, "xp") == 0
    assert int(ex["p_health"][0, 0]) == 10       # refilled to max health
    assert _rpg(ex, 0, "mana") == 9              # refilled (then capped regen)
    # below the level threshold nothing is refilled
    ex, _ = _one(oracle_lib, MANA | LEVEL, ents=ents, xp_per_level=3)
    assert _rpg(ex, 0, "xp") == 1 and int(ex["p_health"][0, 0]) == 4


def test_kill_credit_goes_to_the_killing_blow(oracle_lib):
    """Both players hit one NPC with 2 health for 1 each: the second hit in
    the initiative order kills it and takes the experience."""
    ents = [(1, 0, 2, 2, 10), (2, 0, 4, 2, 10), (3, 0, 3, 2, 2)]
    for seed in range(8):
        ex, evs = _one(oracle_lib, LEVEL, ents=ents, moves=((RIGHT, 4),), seed=seed)
        comb = [e[1] for e in evs[0] if e[0] == 1]
        assert len(comb) == 2 and int(ex["npc_alive"][0]) == 0
        second = comb[1]
        assert _rpg(ex, second - 1, "xp") == 1 and _rpg(ex, 2 - second, "xp") == 0


def test_items_drop_and_pickup(oracle_lib, tmp_path):
    """A dying NPC drops an item on its cell (drop chance 100%); stepping onto
    it takes it: +1 damage (kind 0) or +1 max health and health (kind 1)."""
    ents = [(1, 0, 2, 2, 10), (2, 0, 5, 5, 10), (3, 0, 3, 2, 1)]
    kinds = set()
    for seed in range(12):
        ex, evs = _one(oracle_lib, ITEMS, ents=ents, moves=((RIGHT, STAY),), seed=seed)
        assert int(ex["item_mask"][0, 0]) == 1
        assert int(ex["item_pos"][0, 0]) == 3 | (2 << 8)
        kind = int(ex["item_mask"][1, 0]) & 1
        kinds.add(kind)
        ex, evs = _one(oracle_lib, ITEMS, ents=ents, moves=((RIGHT, STAY), (RIGHT, STAY)),
                       seed=seed)
        assert (ex["p_x"][0, 0], ex["p_y"][0, 0]) == (3, 2)
        assert int(ex["item_mask"][0, 0]) == 0
        assert _rpg(ex, 0, "items") == 1
        assert _rpg(ex, 0, "damage") == 2 + (kind == 0)
        assert _rpg(ex, 0, "max_health") == 10 + (kind == 1)
        assert int(ex["p_health"][0, 0]) == 10 + (kind == 1)
        # no free item spot: the item stays on the floor
        ex, _ = _one(oracle_lib, ITEMS, ents=ents, moves=((RIGHT, STAY), (RIGHT, STAY)),
                     seed=seed, item_slots=0)
        assert int(ex["item_mask"][0, 0]) == 1 and _rpg(ex, 0, "items") == 0
    assert kinds == {0, 1}
    # drop chance 0: nothing drops
    ex, _ = _one(oracle_lib, ITEMS, ents=ents, item_drop_pct=0)
    assert int(ex["item_mask"][0, 0]) == 0


README = 64
DUEL = [(1, 0, 2, 2, 10), (2, 0, 3, 2, 10)]   # player 1 left of player 2
LEFT, DOWN = 4, 3


def _duel(oracle_lib, moves, ents=DUEL, flags=README, **kw):
    return _one(oracle_lib, flags, ents=ents, moves=moves, n_npcs=0, player_damage=5,
                player_armor=1, **kw)


def test_readme_combat_mutual(oracle_lib):
    """Both attack the other's cell: each takes half of 5 - 1 = 4, nobody
    moves, both get combat_cooldown (3) ticks of cooldown."""
    ex, evs = _duel(oracle_lib, ((RIGHT, LEFT),))
    assert ex["p_health"][:, 0].tolist() == [8, 8]
    assert ex["p_x"][:, 0].tolist() == [2, 3]
    assert _rpg(ex, 0, "cooldown") == 3 and _rpg(ex, 1, "cooldown") == 3
    assert evs[0] == [(1, 1, 2, 4), (1, 2, 1, 4)]
    # the next three ticks their attacks are Stays and they cannot defend:
    # player 1 attacking is a Stay, player 2 attacks it (full damage, no stun)
    ex, evs = _duel(oracle_lib, ((RIGHT, LEFT), (RIGHT, LEFT)))
    assert ex["p_health"][:, 0].tolist() == [8, 8]   # both attacks measured as Stays
    assert evs[1] == []
    # cooldown runs out after combat_cooldown ticks
    ex, _ = _duel(oracle_lib, ((RIGHT, LEFT), (STAY, STAY), (STAY, STAY), (STAY, STAY)))
    assert _rpg(ex, 0, "cooldown") == 0
    ex, _ = _duel(oracle_lib, ((RIGHT, LEFT),), combat_cooldown=5)
    assert _rpg(ex, 1, "cooldown") == 5


def test_readme_combat_same_cell(oracle_lib):
    """Both move into one cell: full damage each, nobody moves."""
    ents = [(1, 0, 2, 2, 10), (2, 0, 4, 2, 10)]
    ex, evs = _duel(oracle_lib, ((RIGHT, LEFT),), ents=ents)
    assert ex["p_health"][:, 0].tolist() == [6, 6]
    assert ex["p_x"][:, 0].tolist() == [2, 4]
    assert evs[0] == [(1, 1, 2, 2), (1, 2, 1, 2)]


def test_readme_combat_negation_and_stun(oracle_lib):
    """A attacks B who stays: negated, A is stunned one tick (cannot attack or
    defend); B then attacks the stunned A: full damage."""
    ex, evs = _duel(oracle_lib, ((RIGHT, STAY),))
    assert ex["p_health"][:, 0].tolist() == [10, 10]
    assert _rpg(ex, 0, "cooldown") == 1 and evs[0] == [(1, 1, 2, 1)]
    ex, evs = _duel(oracle_lib, ((RIGHT, STAY), (RIGHT, LEFT)))
    assert ex["p_health"][:, 0].tolist() == [6, 10]
    assert evs[1] == [(1, 2, 1, 1)]
    assert _rpg(ex, 1, "cooldown") == 0            # an undefended hit stuns nobody
    # a healer stays too: its attacker is negated
    ex, _ = _duel(oracle_lib, ((RIGHT, HEAL_MOVE),), flags=README | MANA | HEAL)
    assert int(ex["p_health"][1, 0]) == 10


def test_readme_combat_flee(oracle_lib):
    """A attacks B's cell but B moves away: no damage, A stays."""
    ex, evs = _duel(oracle_lib, ((RIGHT, DOWN),))
    assert ex["p_health"][:, 0].tolist() == [10, 10]
    assert (ex["p_x"][:, 0].tolist(), ex["p_y"][:, 0].tolist()) == ([2, 3], [2, 3])
    assert evs[0][0] == (1, 1, 2, 3)


def test_readme_combat_mana(oracle_lib):
    """Mana joins the readme's damage: half of (4 + 3) = 3 in a mutual attack."""
    ex, _ = _duel(oracle_lib, ((RIGHT, LEFT),), flags=README | MANA)
    assert ex["p_health"][:, 0].tolist() == [7, 7]
    assert _rpg(ex, 0, "mana") == 9 - 3 + 1


def test_rpg_oracle_runs_many_games(oracle_lib):
    """Many random games with every mechanic on: invariants of the attributes."""
    cfg = dict(width=10, height=9, n_npcs=6, npc_health=3, max_ticks=200, flags=MANA | HEAL | LEVEL | ITEMS,
               mana_max=9, mana_regen=1, mana_per_point=1, xp_per_kill=1, xp_per_level=2,
               item_drop_pct=60, item_bonus=2, item_slots=2)
    B = 256
    o = oracle_lib.Oracle(cfg, B, 5, 0)
    o.reset(episode=np.zeros(B, np.int32))
    rs = np.random.RandomState(0)
    picked = xp = 0
    for t in range(300):
        o.step(rs.randint(1, 7, size=(B, 2)).astype(np.int8))
        ex = o.export()
        r = ex["p_rpg"]
        assert (r[0] >= 0).all() and (r[0] <= 9).all()          # mana within the bar
        assert (r[4] <= 2).all()                                  # item spots
        assert (r[2] == 2 + 2 * (r[4] - (r[3] - 10) // 2)).all()  # bonuses = items held
        picked += int(r[4].sum())
        xp += int(r[1].sum())
    assert picked > 0 and xp > 0


# ---------------------------------------------------------------------------
# GPU: the engine against the oracle, bit for bit
# ---------------------------------------------------------------------------
RPG_CASES = {
    # every mechanic, random moves incl. heals, NPC-dense small boards
    "rpg_all_10x9": (dict(width=10, height=9, n_npcs=6, npc_health=3, max_ticks=200,
                          flags=MANA | HEAL | LEVEL | ITEMS, xp_per_level=2, item_drop_pct=60,
                          item_bonus=2, item_slots=2), 2048, 300, 31, 0),
    "rpg_16npc_8x8": (dict(width=8, height=8, n_npcs=16, npc_health=2, max_ticks=100,
                           flags=MANA | LEVEL | ITEMS, mana_max=12, mana_per_point=2,
                           item_drop_pct=100), 2048, 200, 32, 0),
    # separated start (items on player 1's start depth), descents, separation damage
    "rpg_separated": (dict(width=9, height=9, start_mode=2, p1_depth=1, p2_depth=0, n_npcs=3,
                           max_ticks=300, flags=1 | MANA | HEAL | ITEMS, sep_period=4),
                      2048, 300, 33, 0),
    "rpg_c3_64": (dict(width=64, height=64, n_npcs=8, max_ticks=1000,
                       flags=MANA | HEAL | LEVEL | ITEMS), 4096, 400, 34, 0),
    # deadly and cramped: players die in meets the same tick they pick up health
    # items or level up; one item spot; every kill a level
    "rpg_deadly_5x6": (dict(width=5, height=6, n_npcs=5, npc_health=2, player_health=2,
                            max_ticks=0, flags=MANA | LEVEL | ITEMS, mana_max=3,
                            xp_per_level=1, item_drop_pct=90, item_bonus=2, item_slots=1),
                       2048, 300, 36, 0),
    # the readme's combat table, alone and with every other mechanic
    "readme_combat_5x5": (dict(width=5, height=5, n_npcs=2, max_ticks=300, flags=README,
                               player_damage=4), 2048, 300, 37, 0),
    "readme_all_8x7": (dict(width=8, height=7, n_npcs=5, max_ticks=200,
                            flags=README | MANA | HEAL | LEVEL | ITEMS | 1, sep_period=5,
                            start_mode=2, p1_depth=0, p2_depth=1, xp_per_level=2),
                       2048, 300, 38, 0),
    # stock-seed mode with the mechanics (drops keep their Philox block)
    "rpg_stock": (dict(width=10, height=9, n_npcs=4, max_ticks=150, rng=1,
                       flags=MANA | HEAL | LEVEL | ITEMS), 1024, 300, 35, 0),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(RPG_CASES))
def test_rpg_engine_vs_oracle(name, oracle_lib):
    """orx_step_events with random actions 1..6 (heals included): state,
    character attributes, items and every update event against the oracle;
    then orx_rollout (StaircaseBot vs RandomBot) against the oracle's
    policy+step."""
    import torch
    from golden_util import compare_state
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    cfg, B, T, seed, off = RPG_CASES[name]
    dev = torch.device("cuda", 0)
    ora = oracle_lib.Oracle(cfg, B, seed, off, record_events=True)
    ora.reset(episode=np.zeros(B, np.int32))
    eng = BatchedEngine(EnvConfig.from_dict(cfg), B, seed=seed, game_offset=off, device=dev)
    compare_state(eng.snapshot(), ora.export(), ora.K, f"{name} reset")
    rs = np.random.RandomState(seed)
    hi = 7 if cfg["flags"] & HEAL else 6
    n_heal_ev = 0
    for t in range(T):
        a = rs.randint(1, hi, size=(B, 2)).astype(np.int8)
        ora.step(a)
        _, ev, n = eng.step(torch.from_numpy(a).to(dev).contiguous(), events=True)
        if t % 25 == 24 or t == T - 1:
            compare_state(eng.snapshot(), ora.export(), ora.K, f"{name} t={t + 1}")
        ev, n = ev.cpu().numpy(), n.cpu().numpy()
        for g in range(0, B, 7):
            got = [tuple(int(v) for v in r) for r in ev[g, : n[g]]]
            assert got == ora.events(g), (name, t, g, got, ora.events(g))
            n_heal_ev += sum(1 for r in got if r[0] == 5 and r[2] > 0)
    if cfg["flags"] & HEAL:
        assert n_heal_ev > 0
    ex = ora.export()
    assert ex["p_rpg"][1].sum() > 0 if cfg["flags"] & LEVEL else True
    # the fused rollout on the same configuration: the generic form (StaircaseBot
    # vs RandomBot) and the RandomBot-pair form with trajectories (PM 3)
    from optimax_rogue_amd.enums import OBS_FIELDS
    for pol in ((2, 1), (1, 1)):
        ora2 = oracle_lib.Oracle(cfg, B, seed, off)
        ora2.reset(episode=np.zeros(B, np.int32))
        eng2 = BatchedEngine(EnvConfig.from_dict(cfg), B, seed=seed, game_offset=off, device=dev)
        n = T // 3
        obs = torch.zeros((n, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
        act = torch.zeros((n, B, 2), dtype=torch.int8, device=dev)
        for c in range(3):
            want_act = []
            for _ in range(n):
                a = ora2.policy(*pol)
                want_act.append(a)
                ora2.step(a)
            eng2.rollout(n, *pol, obs=obs, act=act)
            compare_state(eng2.snapshot(), ora2.export(), ora2.K, f"{name} rollout {pol} {c}")
            assert np.array_equal(act.cpu().numpy(), np.stack(want_act)), (name, pol, c)
    torch.cuda.synchronize()
