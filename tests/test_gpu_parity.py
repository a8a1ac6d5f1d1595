"""GPU parity: the HIP engine against the reference's golden fixtures and the
C oracle (bit-exact; all state is integer)."""
import os
import numpy as np
import pytest

from golden_util import STATE_KEYS, Fixture, case_names, compare_state

pytestmark = pytest.mark.gpu


def _engine(cfg, n_games, seed, offset=0, reset=True, layouts=None):
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    return BatchedEngine(EnvConfig.from_dict(cfg, layouts=layouts), n_games, seed=seed,
                         game_offset=offset, device=torch.device("cuda", 0), reset=reset)


@pytest.mark.parametrize("name", case_names())
def test_golden_step_by_step(name):
    """policy kernel + step kernel, tick by tick, vs the reference fixtures."""
    import torch
    fx = Fixture(name)
    eng = _engine(fx.cfg, fx.G, fx.seed, fx.game_offset, layouts=fx.layouts)
    compare_state(eng.snapshot(), fx.state(0), fx.K, f"{name} reset")
    for t in range(fx.T):
        a = eng.policy(*fx.policy)
        got = a.cpu().numpy()
        assert np.array_equal(got, fx.actions[t]), f"{name} policy t={t}"
        eng.step(a)
        compare_state(eng.snapshot(), fx.state(t + 1), fx.K, f"{name} t={t + 1}")
    torch.cuda.synchronize()


@pytest.mark.parametrize("name", case_names())
def test_golden_update_events(name):
    """orx_step_events: every tick's update events (type, entity, args, order)
    equal the GameStateUpdate list the reference returned."""
    import torch
    fx = Fixture(name)
    eng = _engine(fx.cfg, fx.G, fx.seed, fx.game_offset, layouts=fx.layouts)
    acts = torch.from_numpy(fx.actions).to(eng.device)
    for t in range(fx.T):
        if fx.stock:
            eng.policy(*fx.policy)   # the bots' draws share the game's random stream
        _, ev, n = eng.step(acts[t].contiguous(), events=True)
        ev, n = ev.cpu().numpy(), n.cpu().numpy()
        for g in range(fx.G):
            got = [tuple(int(v) for v in r) for r in ev[g, : n[g]]]
            assert got == fx.events(t, g), (name, t, g, got, fx.events(t, g))
    compare_state(eng.snapshot(), fx.state(fx.T), fx.K, f"{name} final")


@pytest.mark.parametrize("name", case_names())
def test_golden_step_given_actions(name):
    """step kernel driven by the fixture's recorded actions (uploaded once)."""
    import torch
    fx = Fixture(name)
    eng = _engine(fx.cfg, fx.G, fx.seed, fx.game_offset, layouts=fx.layouts)
    acts = torch.from_numpy(fx.actions).to(eng.device)
    for t in range(fx.T):
        if fx.stock:
            eng.policy(*fx.policy)
        eng.step(acts[t].contiguous())
    compare_state(eng.snapshot(), fx.state(fx.T), fx.K, f"{name} final")


@pytest.mark.parametrize("name", case_names())
def test_golden_rollout(name):
    """fused rollout kernel: every tick's observation vs the fixtures."""
    import torch
    from optimax_rogue_amd.enums import OBS_FIELDS
    fx = Fixture(name)
    eng = _engine(fx.cfg, fx.G, fx.seed, fx.game_offset, layouts=fx.layouts)
    # split in two launches to exercise state hand-over between launches
    t1 = fx.T // 3
    obs = torch.zeros((fx.T, len(OBS_FIELDS), fx.G), dtype=torch.int32, device=eng.device)
    act = torch.zeros((fx.T, fx.G, 2), dtype=torch.int8, device=eng.device)
    eng.rollout(t1, *fx.policy, obs=obs[:t1], act=act[:t1])
    eng.rollout(fx.T - t1, *fx.policy, obs=obs[t1:], act=act[t1:])
    o = obs.cpu().numpy()
    assert np.array_equal(act.cpu().numpy(), fx.actions)
    for t in range(fx.T):
        s = fx.state(t + 1)
        want = np.stack([s["p_x"][0], s["p_y"][0], s["p_depth"][0], s["p_health"][0],
                         s["p_x"][1], s["p_y"][1], s["p_depth"][1], s["p_health"][1],
                         s["tick"], s["status"], s["st_x"][0], s["st_y"][0], s["st_x"][1],
                         s["st_y"][1]])
        assert np.array_equal(o[t], want), f"{name} obs t={t + 1}"
    compare_state(eng.snapshot(), fx.state(fx.T), fx.K, f"{name} final")


def _bank(W, H, L, seed, stairs=(1,)):
    """Explicit-grid layouts for the large oracle cases (walls ~20%, open edges
    on even layouts, n staircases)."""
    rs = np.random.RandomState(seed)
    out = []
    for li in range(L):
        t = np.ones((W, H), np.uint8)
        t[[0, -1], :] = 2
        t[:, [0, -1]] = 2
        if li % 2 == 0:
            t[0, 1:H - 1] = 1
        inner = rs.rand(W, H) < 0.2
        inner[[0, -1], :] = False
        inner[:, [0, -1]] = False
        t[inner] = 2
        g = np.argwhere(t == 1)
        for j in rs.choice(len(g), stairs[li % len(stairs)], replace=False):
            t[tuple(g[j])] = 3
        out.append(t)
    return np.stack(out)


ORACLE_CASES = {
    "c2_random_32": (dict(width=32, height=32), (1, 1), 4096, 400, 2),
    "npc_small_unused": (dict(width=7, height=6, n_npcs=5, despawn=2, max_ticks=90), (1, 2),
                         4096, 300, 11),
    "separated_stairs": (dict(width=9, height=9, start_mode=2, p1_depth=4, p2_depth=1,
                              n_npcs=3, max_ticks=200), (2, 2), 2048, 400, 12),
    "duel_4": (dict(width=4, height=5, max_ticks=0), (1, 1), 4096, 300, 13),
    "c5_stairs_128": (dict(width=128, height=128), (2, 2), 1024, 600, 5),
    "npc16_8x8": (dict(width=8, height=8, n_npcs=16, npc_health=2, max_ticks=50), (1, 1), 2048,
                  200, 14),
    # explicit-grid dungeon bank (16 layouts), NPCs, both bots, both despawn rules
    "bank_64_npc": (dict(width=64, height=64, n_npcs=8, max_ticks=300), (1, 1), 2048, 400, 15),
    "bank_stairs_unused": (dict(width=12, height=10, n_npcs=2, max_ticks=200, despawn=2), (2, 1),
                           2048, 400, 16),
    # a bank too large for the rollout's LDS staging (64 x 36 x 36 tiles =
    # 81 KiB > 64 KiB): the rollout reads the tiles from global memory
    # (bank_64_npc, exactly 64 KiB, is staged)
    "bank_big_global": (dict(width=36, height=36, n_npcs=4, max_ticks=200), (2, 1), 2048, 300,
                        26),
    # a StaircaseBot descending into a 5x4 depth a RandomBot walks: the
    # rollout's descend-into-the-other's-depth path in both drawn orders
    "desc_meet_5x4": (dict(width=5, height=4, start_mode=2, p1_depth=2, p2_depth=1,
                           max_ticks=200), (1, 2), 2048, 200, 25),
    # Unused despawn with a separated start: player 1 leaves the NPCs' depth,
    # it is despawned, and player 2 descends into its regeneration, whose
    # staircase may lie under an NPC (attacked, not descended through)
    "npc_stair_unused_sep": (dict(width=6, height=6, start_mode=2, p1_depth=1, p2_depth=0,
                                  n_npcs=10, despawn=2, max_ticks=300), (2, 2), 4096, 400, 48),
    "npc_stair_unused_bank": (dict(width=8, height=7, start_mode=2, p1_depth=1, p2_depth=0,
                                   n_npcs=9, despawn=2, max_ticks=300), (2, 2), 4096, 400, 49),
    # dense NPCs (K > 16): the occupancy-grid form, from crowded to packed
    "npc_dense_40_16x16": (dict(width=16, height=16, n_npcs=40, npc_health=2, max_ticks=150),
                           (1, 2), 2048, 300, 40),
    "npc_dense_200_20x20": (dict(width=20, height=20, n_npcs=200, npc_health=1, max_ticks=80,
                                 despawn=2), (1, 1), 1024, 200, 41),
    "npc_dense_64_c3": (dict(width=64, height=64, n_npcs=64, max_ticks=1000), (1, 1), 4096, 400,
                        42),
    "npc_dense_bank": (dict(width=12, height=10, n_npcs=24, max_ticks=200, start_mode=2,
                            p1_depth=1, p2_depth=0), (2, 1), 2048, 300, 43),
    "npc_dense_stock": (dict(width=10, height=9, n_npcs=20, despawn=2, max_ticks=150, rng=1),
                        (1, 2), 1024, 300, 44),
    # W * H = 99: the game rows of the grid start at every byte offset mod 4
    "npc_dense_odd_9x11": (dict(width=9, height=11, n_npcs=21, npc_health=1, max_ticks=40),
                           (1, 1), 1023, 200, 47),
    "npc_dense_rpg": (dict(width=12, height=12, n_npcs=30, npc_health=2, max_ticks=200,
                           flags=4 | 16 | 64, xp_per_level=2), (1, 1), 2048, 300, 45),
    # build extensions (readme-only mechanics, parity unpinned: engine vs oracle)
    "ext_separation": (dict(width=9, height=9, start_mode=2, p1_depth=0, p2_depth=2, n_npcs=2,
                            max_ticks=300, flags=1, sep_period=4), (2, 1), 2048, 400, 17),
    "ext_double_death": (dict(width=4, height=5, max_ticks=0, player_health=1, flags=3,
                              sep_period=2), (1, 1), 2048, 200, 18),
    # stock-seed mode (MT19937 per game, reference call order)
    "stock_npc_unused": (dict(width=10, height=9, n_npcs=4, despawn=2, max_ticks=150, rng=1),
                         (1, 2), 2048, 400, 19),
    "stock_c5_stairs": (dict(width=128, height=128, rng=1), (2, 2), 1024, 600, 20),
    "stock_bank_separated": (dict(width=12, height=10, n_npcs=2, start_mode=2, p1_depth=3,
                                  p2_depth=0, max_ticks=200, rng=1), (2, 1), 2048, 400, 21),
    "stock_ext": (dict(width=4, height=5, max_ticks=0, player_health=1, flags=3, sep_period=2,
                       rng=1), (1, 1), 2048, 200, 23),
    # moving NPCs (npc_policy: 1 RANDOM, 2 CHASE -- the enemy AI behind
    # Updater.decide_npc_move): register and dense NPCs, both despawn rules,
    # a Separated start whose NPC depth is left and re-entered, a bank, stock
    # seeding, the build extensions
    "mnpc_random_c3": (dict(width=64, height=64, n_npcs=8, max_ticks=300, npc_policy=1), (1, 1),
                       2048, 400, 60),
    "mnpc_chase_dense": (dict(width=16, height=14, n_npcs=40, npc_health=2, max_ticks=150,
                              npc_policy=2), (2, 1), 1024, 300, 61),
    "mnpc_random_dense_unused": (dict(width=12, height=12, n_npcs=30, npc_health=2, despawn=2,
                                      max_ticks=120, npc_policy=1), (2, 2), 1024, 300, 62),
    "mnpc_stairs_unused": (dict(width=10, height=9, n_npcs=12, despawn=2, max_ticks=100,
                                npc_policy=1), (2, 2), 2048, 300, 63),
    "mnpc_separated": (dict(width=9, height=9, start_mode=2, p1_depth=3, p2_depth=0, n_npcs=6,
                            max_ticks=200, npc_policy=1), (2, 1), 2048, 300, 64),
    "mnpc_chase_bank": (dict(width=12, height=10, n_npcs=10, max_ticks=150, npc_policy=2),
                        (1, 2), 2048, 300, 65),
    "mnpc_stock": (dict(width=8, height=8, n_npcs=6, max_ticks=80, rng=1, npc_policy=1), (1, 2),
                   1024, 240, 66),
    "mnpc_ext": (dict(width=8, height=8, start_mode=2, p1_depth=0, p2_depth=1, n_npcs=9,
                      npc_damage=2, max_ticks=0, flags=3, sep_period=3, npc_policy=2), (2, 1),
                 2048, 300, 67),
}
ORACLE_BANKS = {"bank_64_npc": (64, 64, 16, 21, (1,)), "bank_stairs_unused": (12, 10, 5, 22, (1, 3)),
                "npc_dense_bank": (12, 10, 6, 46, (1, 2)),
                "bank_big_global": (36, 36, 64, 27, (1, 2)),
                "stock_bank_separated": (12, 10, 7, 24, (1, 2)),
                "npc_stair_unused_bank": (8, 7, 6, 50, (1, 2)),
                "mnpc_chase_bank": (12, 10, 5, 51, (1, 2))}


@pytest.mark.parametrize("name", sorted(ORACLE_CASES))
def test_vs_oracle_large(name, oracle_lib):
    """thousands of games: engine (policy+step and rollout) vs the C oracle."""
    import torch
    cfg, pol, B, T, seed = ORACLE_CASES[name]
    lay = _bank(*ORACLE_BANKS[name]) if name in ORACLE_BANKS else None
    ora = oracle_lib.Oracle(cfg, B, seed, 0, layouts=lay)
    ora.reset(episode=np.zeros(B, np.int32))
    eng = _engine(cfg, B, seed, layouts=lay)
    eng2 = _engine(cfg, B, seed, layouts=lay)
    compare_state(eng.snapshot(), ora.export(), ora.K, f"{name} reset")
    chunk = T // 4
    for c in range(4):
        for _ in range(chunk):
            a = ora.policy(*pol)
            ora.step(a)
            eng.step(eng.policy(*pol))
        eng2.rollout(chunk, *pol)
        want = ora.export()
        compare_state(eng.snapshot(), want, ora.K, f"{name} step chunk {c}")
        compare_state(eng2.snapshot(), want, ora.K, f"{name} rollout chunk {c}")
        for e in (eng, eng2):
            if e.npc_grid is not None:
                _check_npc_grid(e, want, f"{name} chunk {c}")
    torch.cuda.synchronize()


def _check_npc_grid(eng, snap, where):
    """Dense NPCs: the HBM occupancy grid holds slot + 1 exactly on the live
    NPCs' cells and 0 elsewhere."""
    from optimax_rogue_amd.enums import npc_alive_bits
    K, H = eng.K, int(eng.cfg.height)
    grid = eng.npc_grid.cpu().numpy()
    want = np.zeros_like(grid)
    live = npc_alive_bits(snap["npc_alive"], K)
    pos = np.asarray(snap["npc_pos"]).astype(np.int64)
    k, g = np.nonzero(live)
    want[g, (pos[k, g] & 0xFF) * H + (pos[k, g] >> 8)] = k + 1
    assert np.array_equal(grid, want), where


def test_ext_events_vs_oracle(oracle_lib):
    """Separation-damage EntityHealthUpdate records and random double-death
    outcomes: orx_step_events against the oracle, tick by tick."""
    import torch
    cfg = dict(width=6, height=6, start_mode=2, p1_depth=1, p2_depth=0, max_ticks=120,
               flags=3, sep_period=2, n_npcs=1)
    B = 512
    ora = oracle_lib.Oracle(cfg, B, 19, 0, record_events=True)
    ora.reset(episode=np.zeros(B, np.int32))
    eng = _engine(cfg, B, 19)
    seen_health = 0
    for t in range(150):
        a = ora.policy(2, 1)
        ora.step(a)
        _, ev, n = eng.step(torch.from_numpy(a).to(eng.device).contiguous(), events=True)
        ev, n = ev.cpu().numpy(), n.cpu().numpy()
        for g in range(B):
            got = [tuple(int(v) for v in r) for r in ev[g, : n[g]]]
            assert got == ora.events(g), (t, g)
            seen_health += sum(1 for r in got if r[0] == 5)
    compare_state(eng.snapshot(), ora.export(), 1, "ext final")
    assert seen_health > 100


def test_sharding_invariance():
    """a game's trajectory depends on its global id only (game_offset)."""
    cfg = dict(width=10, height=10, n_npcs=3, max_ticks=80)
    full = _engine(cfg, 3000, 21)
    a = _engine(cfg, 1000, 21, 0)
    b = _engine(cfg, 2000, 21, 1000)
    for e in (full, a, b):
        e.rollout(250, 1, 2)
    sf, sa, sb = full.snapshot(), a.snapshot(), b.snapshot()
    for k in STATE_KEYS:
        axis = sf[k].ndim - 1
        assert np.array_equal(sf[k], np.concatenate([sa[k], sb[k]], axis=axis)), k


def test_loaded_library_is_the_trees_kernel():
    """The liborx.so these tests run was built from this tree's sources."""
    from optimax_rogue_amd import _lib, build
    _engine(dict(width=8, height=8), 1, 0)
    assert _lib.build_id() == build.source_id()


@pytest.mark.parametrize("which", ["c5_sep", "npc_dense", "c3"])
def test_rollout_games_per_wave_invariance(which, monkeypatch):
    """Results do not depend on how many games a rollout wave carries
    (orx_rollout_lanes; ORX_ROLLOUT_LANES forces it), FAST and plain kernels,
    with trajectories, across resets, descends and NPC hits."""
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.enums import EXT_SEPARATION_DAMAGE, OBS_FIELDS
    if which == "c5_sep":
        cfg = dict(EnvConfig.c5().to_dict(), width=16, height=12, max_ticks=90,
                   flags=EXT_SEPARATION_DAMAGE, sep_period=4)
        pol, B, T = (2, 1), 3001, 300
    elif which == "npc_dense":
        cfg = dict(width=8, height=8, n_npcs=16, max_ticks=60)
        pol, B, T = (1, 2), 2053, 200
    else:
        cfg = dict(EnvConfig.c3().to_dict(), max_ticks=100)
        pol, B, T = (1, 1), 4099, 150
    ref = None
    for lanes in (64, 32, 8, 1):
        monkeypatch.setenv("ORX_ROLLOUT_LANES", str(lanes))
        e = _engine(cfg, B, 11, 7)
        assert e.rollout_lanes() == lanes
        obs = torch.zeros((T, len(OBS_FIELDS), B), dtype=torch.int32, device=e.device)
        act = torch.zeros((T, B, 2), dtype=torch.int8, device=e.device)
        e.rollout(T // 2, *pol, obs=obs, act=act)
        e.rollout(T - T // 2, *pol, obs=obs[T // 2:], act=act[T // 2:])
        got = (e.snapshot(), obs.cpu().numpy(), act.cpu().numpy())
        if ref is None:
            ref = got
            continue
        for k in STATE_KEYS:
            assert np.array_equal(got[0][k], ref[0][k]), (lanes, k)
        assert np.array_equal(got[1], ref[1]) and np.array_equal(got[2], ref[2]), lanes
    assert ref[0]["ep_count"].sum() > 0


@pytest.mark.parametrize("n_streams", [2, 3])
def test_stream_shards_equal_one_engine(n_streams):
    """StreamShardedEngine (the bench's per-stream shards) computes exactly
    what one BatchedEngine over the whole batch does: state and trajectory."""
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import StreamShardedEngine
    from optimax_rogue_amd.enums import OBS_FIELDS
    cfg = dict(EnvConfig.c3().to_dict(), max_ticks=100)
    B, T = 5001, 130
    one = _engine(cfg, B, 3, 11)
    obs = torch.zeros((T, len(OBS_FIELDS), B), dtype=torch.int32, device=one.device)
    act = torch.zeros((T, B, 2), dtype=torch.int8, device=one.device)
    one.rollout(T, 1, 1, obs=obs, act=act)
    sh = StreamShardedEngine(EnvConfig.from_dict(cfg), B, seed=3, game_offset=11,
                             device=one.device, n_streams=n_streams)
    so, sa = sh.trajectory_buffers(T)
    go = sh.rollout_launcher(T, 1, 1, obs=so, act=sa)
    sh.fork()
    go()
    sh.join()
    a, b = one.snapshot(), sh.snapshot()
    for k in STATE_KEYS:
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(obs.cpu().numpy(), torch.cat(so, dim=2).cpu().numpy())
    assert np.array_equal(act.cpu().numpy(), torch.cat(sa, dim=1).cpu().numpy())
    assert a["ep_count"].sum() >= B


def test_engines_sharing_shard_streams():
    """Two StreamShardedEngines alive at once share the process's shard
    streams (engine.shard_streams); their launches interleave on them and
    each still computes what its own single engine does."""
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import StreamShardedEngine
    from optimax_rogue_amd.enums import OBS_FIELDS
    cfg = dict(EnvConfig.c3().to_dict(), max_ticks=60)
    B, T = 3000, 70
    dev = torch.device("cuda", 0)
    engs = [StreamShardedEngine(EnvConfig.from_dict(cfg), B, seed=s, device=dev, n_streams=2)
            for s in (4, 9)]
    assert all(x is y for x, y in zip(engs[0].streams, engs[1].streams))
    bufs = [e.trajectory_buffers(T) for e in engs]
    gos = [e.rollout_launcher(T, 1, 1, obs=o, act=a) for e, (o, a) in zip(engs, bufs)]
    for e in engs:
        e.fork()
    for _ in range(2):
        for go in gos:
            go()
    for e in engs:
        e.join()
    for s, e, (so, sa) in zip((4, 9), engs, bufs):
        one = _engine(cfg, B, s)
        obs = torch.zeros((T, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
        act = torch.zeros((T, B, 2), dtype=torch.int8, device=dev)
        one.rollout(T, 1, 1, obs=obs, act=act)
        one.rollout(T, 1, 1, obs=obs, act=act)
        a, b = one.snapshot(), e.snapshot()
        for k in STATE_KEYS:
            assert np.array_equal(a[k], b[k]), (s, k)
        assert np.array_equal(obs.cpu().numpy(), torch.cat(so, dim=2).cpu().numpy()), s
        assert np.array_equal(act.cpu().numpy(), torch.cat(sa, dim=1).cpu().numpy()), s


@pytest.mark.parametrize("pol", [(1, 1), (2, 2)])
def test_bank_rollout_forms_agree(pol, monkeypatch):
    """A dungeon bank through the trajectory-specialized rollout (obs and act:
    buffer stores, LDS-staged tiles), the generic one (act only) and with the
    LDS staging disabled: identical states and observation rows."""
    import torch
    from optimax_rogue_amd import DungeonBank
    from optimax_rogue_amd.enums import OBS_FIELDS
    bank = DungeonBank.random(40, 30, 12, seed=5, n_stairs=2)
    cfg = dict(width=40, height=30, n_npcs=4, max_ticks=150)
    B, T = 3001, 200
    res = []
    for no_lds, with_obs in (("", True), ("", False), ("1", True)):
        if no_lds:
            monkeypatch.setenv("ORX_NO_LDS_TILES", "1")
        else:
            monkeypatch.delenv("ORX_NO_LDS_TILES", raising=False)
        e = _engine(cfg, B, 9, layouts=bank.layouts)
        obs = torch.zeros((T, len(OBS_FIELDS), B), dtype=torch.int32, device=e.device)
        act = torch.zeros((T, B, 2), dtype=torch.int8, device=e.device)
        e.rollout(T, *pol, obs=obs if with_obs else None, act=act)
        res.append((e.snapshot(), obs.cpu().numpy() if with_obs else None, act.cpu().numpy()))
    for got in res[1:]:
        for k in STATE_KEYS:
            assert np.array_equal(got[0][k], res[0][0][k]), k
        assert np.array_equal(got[2], res[0][2])
    assert np.array_equal(res[2][1], res[0][1])
    assert res[0][0]["ep_count"].sum() > 0 and res[0][0]["counters"][1].sum() > 0


def test_rollout_equals_step_c3():
    """C3 shape (B=65536, 64x64, K=8): fused rollout == per-tick policy+step."""
    from optimax_rogue_amd import EnvConfig
    cfg = EnvConfig.c3().to_dict()
    e1 = _engine(cfg, 65536, 3)
    e2 = _engine(cfg, 65536, 3)
    for _ in range(64):
        e1.step(e1.policy(1, 1))
    e2.rollout(64, 1, 1)
    s1, s2 = e1.snapshot(), e2.snapshot()
    for k in STATE_KEYS:
        assert np.array_equal(s1[k], s2[k]), k


def _invariants(s, cfg):
    W, H = cfg["width"], cfg["height"]
    for p in range(2):
        assert (s["p_x"][p] >= 1).all() and (s["p_x"][p] <= W - 2).all()
        assert (s["p_y"][p] >= 1).all() and (s["p_y"][p] <= H - 2).all()
        assert (s["st_x"][p] >= 1).all() and (s["st_x"][p] <= W - 3).all()
        assert (s["st_y"][p] >= 1).all() and (s["st_y"][p] <= H - 3).all()
        # a player never stands on its staircase (it would have descended)
        assert not ((s["p_x"][p] == s["st_x"][p]) & (s["p_y"][p] == s["st_y"][p])).any()
    same = ((s["p_depth"][0] == s["p_depth"][1]) & (s["p_x"][0] == s["p_x"][1])
            & (s["p_y"][0] == s["p_y"][1]))
    assert not same.any(), "two players on one cell"
    both_same_depth = s["p_depth"][0] == s["p_depth"][1]
    assert np.array_equal(s["st_x"][0][both_same_depth], s["st_x"][1][both_same_depth])
    assert (s["p_health"] <= cfg.get("player_health", 10)).all()
    assert set(np.unique(s["status"]).tolist()) <= {1, 2, 3, 4}


def _obs_rows(ex):
    """The 14-field observation rows (OBS_FIELDS order) of an oracle export:
    int32 [14, games]."""
    return np.stack([ex["p_x"][0], ex["p_y"][0], ex["p_depth"][0], ex["p_health"][0],
                     ex["p_x"][1], ex["p_y"][1], ex["p_depth"][1], ex["p_health"][1],
                     ex["tick"], ex["status"], ex["st_x"][0], ex["st_y"][0],
                     ex["st_x"][1], ex["st_y"][1]]).astype(np.int32)


def _replay(ora, n_ticks, pol=(1, 1)):
    """n_ticks of policy + step on the oracle: (act [T, games, 2], obs [T, 14, games])."""
    acts, obs = [], []
    for _ in range(n_ticks):
        a = ora.policy(*pol)
        ora.step(a)
        acts.append(a)
        obs.append(_obs_rows(ora.export()))
    return np.stack(acts), np.stack(obs)


def test_c3_full_size_properties(oracle_lib):
    """B=65536 at 64x64 with K=8, one 1000-tick launch WITH the trajectory
    outputs (so the PM=1 RandomBot/buffer-store form at 64 games per wave):
    invariants after it, and a sample of games replayed on the oracle by
    global id -- every tick's observation row and action pair, and the final
    state."""
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.enums import OBS_FIELDS
    cfg = EnvConfig.c3().to_dict()
    B, T = 65536, 1000
    eng = _engine(cfg, B, 3)
    obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=eng.device)
    act = torch.empty((T, B, 2), dtype=torch.int8, device=eng.device)
    eng.rollout(T, 1, 1, obs=obs, act=act)
    s = eng.snapshot()
    _invariants(s, cfg)
    assert s["ep_count"].sum() >= B  # max_ticks 1000 -> every game finished once
    rng = np.random.default_rng(0)
    gids = np.sort(rng.choice(B, 48, replace=False))
    idx = torch.from_numpy(gids).to(eng.device)
    g_obs = obs.index_select(2, idx).cpu().numpy()
    g_act = act.index_select(1, idx).cpu().numpy()
    del obs, act
    for j, gid in enumerate(gids):
        ora = oracle_lib.Oracle(cfg, 1, 3, int(gid))
        ora.reset(episode=np.zeros(1, np.int32))
        w_act, w_obs = _replay(ora, T)
        assert np.array_equal(g_act[:, j:j + 1], w_act), f"gid {gid} actions"
        assert np.array_equal(g_obs[:, :, j:j + 1], w_obs), f"gid {gid} observation rows"
        got = {k: (v[..., gid:gid + 1]) for k, v in s.items()}
        compare_state(got, ora.export(), 8, f"gid {gid}")


def _timed_form_vs_oracle(oracle_lib, eng, parts, obs, act, launch, cfg, pol, seed, T, L,
                          starts, offset=0, compact=False, win=8, whole=False):
    """Runs ``launch`` (a pre-bound rollout launcher over ``parts``, each with
    its obs/act buffers) L times as bench.py issues it, and replays
    ``win``-game windows of consecutive games starting at local index
    ``starts`` (global id = ``offset`` + local) on the oracle tick by tick:
    every tick's 14-field observation row and both actions of every launch,
    and the whole state after each launch (``compact``: the launch writes
    ORX_OBS_COMPACT rows, decoded before the comparison).  ``whole``: also
    every game of the batch against a threaded oracle over all of it (its
    whole state after every launch).  Returns the last snapshot and the
    sampled local indices."""
    import torch
    from oracle_pool import OraclePool
    dev = parts[0].device
    gids = np.concatenate([np.arange(s, s + win) for s in starts]) + offset
    oras = []
    for s in starts:
        o = oracle_lib.Oracle(cfg.to_dict(), win, seed, s + offset, layouts=cfg.layouts)
        o.reset(episode=np.zeros(win, np.int32))
        oras.append(o)
    B = sum(e.B for e in parts)
    pool = OraclePool(oracle_lib, cfg.to_dict(), B, seed, offset,
                      layouts=cfg.layouts) if whole else None
    # per shard: which sampled ids it holds, at which local index
    sel = []
    for e in parts:
        loc = gids - e.game_offset
        m = (loc >= 0) & (loc < e.B)
        sel.append((np.nonzero(m)[0], torch.from_numpy(loc[m]).to(dev)))
    sharded = hasattr(eng, "fork")
    for n in range(L):
        if sharded:
            eng.fork()
        launch()
        if sharded:
            eng.join()
        torch.cuda.synchronize()
        g_obs = np.zeros((T, 14, len(gids)), np.int32)
        g_act = np.zeros((T, len(gids), 2), np.int8)
        for (pos, li), o, a in zip(sel, obs, act):
            rows = o.index_select(2, li)
            if compact:
                from optimax_rogue_amd.engine import decode_compact
                rows = decode_compact(rows)
            g_obs[:, :, pos] = rows.cpu().numpy()
            g_act[:, pos] = a.index_select(1, li).cpu().numpy()
        snap = eng.snapshot()
        for w, (s, ora) in enumerate(zip(starts, oras)):
            cols = slice(win * w, win * w + win)
            w_act, w_obs = _replay(ora, T, pol)
            where = f"launch {n} ids {s}..{s + win - 1}"
            assert np.array_equal(g_act[:, cols], w_act), f"{where}: actions"
            assert np.array_equal(g_obs[:, :, cols], w_obs), f"{where}: observation rows"
            got = {k: v[..., s:s + win] for k, v in snap.items()}
            compare_state(got, ora.export(), cfg.n_npcs, f"{where}: state")
        if pool is not None:   # every game of the batch
            pool.rollout(*pol, T)
            compare_state(snap, pool.export(), cfg.n_npcs, f"launch {n}: all {B} games")
    return snap, gids - offset


def _window_starts(B, shard_size, n_random, seed):
    """Both ends of every shard plus n_random 8-aligned windows inside."""
    ends = []
    for off in range(0, B, shard_size):
        ends += [off, off + shard_size - 8]
    rng = np.random.default_rng(seed)
    pool = np.setdiff1d(np.arange(8, B - 8, 8), ends)
    return sorted(set(ends) | {int(x) for x in rng.choice(pool, n_random, replace=False)})


@pytest.mark.parametrize("offset", [0, 458752])
def test_bench_timed_path_vs_oracle(offset, oracle_lib):
    """bench.py's timed path exactly: StreamShardedEngine(C3, 65,536 games,
    seed 3, two stream shards of 32,768) launched through rollout_launcher
    with both trajectory buffers -- pair_rollout_kernel<8, 1, 2, false> (two
    lanes per game, register NPCs, RandomBots, nontemporal stores) at 32
    games per wave -- for 9 back-to-back 128-tick launches (1,152 ticks: every
    game crosses the max_ticks-1000 autoreset), as bench.py issues them (fork,
    launches, join); at game offset 0 (rank 0) and 458,752 (rank 7 of C4's
    eight 65,536-game ranks).  Every one of the 65,536 games: its whole state
    after each launch against a threaded C oracle over the batch; and 4,096
    games -- four windows of 1,024 consecutive global ids at both ends of
    each shard -- replayed tick by tick: every tick's 14-field observation
    row and both actions of every launch (updater.py:76-162,
    randombot.py:20-21)."""
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import StreamShardedEngine
    cfg = EnvConfig.c3()
    B, T, L, seed = 65536, 128, 9, 3
    dev = torch.device("cuda", 0)
    eng = StreamShardedEngine(cfg, B, seed=seed, game_offset=offset, device=dev, n_streams=2)
    assert [e.B for e in eng.parts] == [32768, 32768]
    assert [e.game_offset for e in eng.parts] == [offset, offset + 32768]
    sh = eng.rollout_shape(1, 1)
    assert (sh["games_per_wave"], sh["lanes_per_game"], sh["nontemporal"]) == (32, 2, True)
    obs, act = eng.trajectory_buffers(T)
    launch = eng.rollout_launcher(T, 1, 1, obs=obs, act=act)
    starts = [0, 32768 - 1024, 32768, 65536 - 1024]
    snap, gids = _timed_form_vs_oracle(oracle_lib, eng, eng.parts, obs, act, launch, cfg,
                                       (1, 1), seed, T, L, starts, offset, win=1024,
                                       whole=True)
    assert len(gids) == 4096
    # every game went through the max_ticks autoreset in the timed form
    assert (snap["ep_count"] >= 1).all() and (snap["episode"] >= 1).all()


@pytest.mark.parametrize("sep", [0, 1])
def test_bench_c5_share_stream_shards_vs_oracle(sep, oracle_lib):
    """bench.py's C5 line at the 8-GPU share as it is timed since round 4:
    StreamShardedEngine(C5, 16,384 games, seed 5, two stream shards of 8,192)
    -- pair_rollout_kernel<0, 2, 0, SEP> at 8 games per wave -- for 9
    back-to-back 128-tick launches (fork, launches, join), separation damage
    off (reference semantics) and on; sampled games replayed on the oracle
    tick by tick, and every game's state after every launch against a
    threaded oracle over the batch (staircasebot.py:9-21, updater.py:76-162)."""
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import StreamShardedEngine
    from optimax_rogue_amd.enums import EXT_SEPARATION_DAMAGE
    cfg = EnvConfig.c5()
    if sep:
        cfg.flags, cfg.sep_period = EXT_SEPARATION_DAMAGE, 8
    B, T, L, seed = 16384, 128, 9, 5
    eng = StreamShardedEngine(cfg, B, seed=seed, game_offset=0, device=torch.device("cuda", 0),
                              n_streams=2)
    assert [e.B for e in eng.parts] == [8192, 8192]
    sh = eng.rollout_shape(2, 2)
    assert (sh["games_per_wave"], sh["lanes_per_game"], sh["nontemporal"]) == (8, 2, False)
    obs, act = eng.trajectory_buffers(T)
    launch = eng.rollout_launcher(T, 2, 2, obs=obs, act=act)
    starts = _window_starts(B, 8192, 6, 17)
    snap, gids = _timed_form_vs_oracle(oracle_lib, eng, eng.parts, obs, act, launch, cfg,
                                       (2, 2), seed, T, L, starts, whole=True)
    assert (snap["ep_count"][gids] >= 1).all()
    assert snap["counters"][1][gids].sum() > 100   # the StaircaseBots went deep


# bench.py's sharded extras at their exact timed shapes (bench.extras:
# rollout_rate(..., streams=2), seed 5): StreamShardedEngine over two stream
# shards, 9 back-to-back 128-tick launches (fork, launches, join)
SHARDED_EXTRAS = {
    # the dungeon bank: 16 random 64x64 layouts (bench.py: DungeonBank.random(
    # 64, 64, 16, seed=7)) = exactly 64 KiB of tiles staged in LDS, the
    # paired pair_rollout_kernel<8, 1, 2, false, false, true> at 32 per wave
    "bank": ("bank", 65536, 2, (1, 1), 65536),
    # C3 with the character mechanics (EXT_RPG): pair_rollout_kernel<8, 3, ...>
    "c3_rpg": ("c3_rpg", 65536, 2, (1, 1), 0),
    # C5's 131,072 games on one GPU as two 65,536-game shards (round 5: the
    # paired StaircaseBot form at 32 games per wave), separation damage off / on
    "c5_131072_sep_off": ("c5", 131072, 2, (2, 2), 0),
    "c5_131072_sep_on": ("c5sep", 131072, 2, (2, 2), 0),
    # round 5: a RandomBot against a StaircaseBot on C3 (the c3_mixed extra,
    # pair_rollout_kernel<8, 4, ...>: the mixed paired form)
    "c3_mixed": ("c3", 65536, 2, (1, 2), 0),
}


def _extras_cfg(which):
    from optimax_rogue_amd import DungeonBank, EnvConfig
    from optimax_rogue_amd.enums import EXT_RPG, EXT_SEPARATION_DAMAGE
    if which == "bank":
        bank = DungeonBank.random(64, 64, 16, seed=7)
        return EnvConfig(width=64, height=64, n_npcs=8, layouts=bank.layouts)
    if which == "c3_rpg":
        return EnvConfig(width=64, height=64, n_npcs=8, flags=EXT_RPG)
    if which == "c3":
        return EnvConfig.c3()
    cfg = EnvConfig.c5()
    if which == "c5sep":
        cfg.flags, cfg.sep_period = EXT_SEPARATION_DAMAGE, 8
    return cfg


@pytest.mark.parametrize("name", sorted(SHARDED_EXTRAS))
def test_bench_sharded_extras_vs_oracle(name, oracle_lib):
    """The bench's two-stream-shard extras in the exact form they are timed:
    the shape (two lanes per game, 32 games per wave, nontemporal stores,
    256-thread workgroups, the bank's 65,536 B LDS stage -- the staging loop's
    boundary), then 9 launches of 128 ticks with >= 64 sampled games (8-game
    windows incl. both ends of each shard) replayed on the oracle: every
    tick's observation row, both actions and the state after each launch --
    and every game's state after each launch against a threaded oracle over
    the whole batch
    (worldgen.py:9-26, world.py:41-66 for the bank; readme.md:44-48,69-74 for
    the character mechanics, parity unpinned; staircasebot.py:9-21)."""
    import torch
    from optimax_rogue_amd.engine import StreamShardedEngine
    which, B, streams, pol, lds = SHARDED_EXTRAS[name]
    cfg = _extras_cfg(which)
    T, L, seed = 128, 9, 5
    eng = StreamShardedEngine(cfg, B, seed=seed, game_offset=0, device=torch.device("cuda", 0),
                              n_streams=streams)
    sh = eng.rollout_shape(*pol)
    assert (sh["games_per_wave"], sh["lanes_per_game"], sh["nontemporal"],
            sh["threads_per_block"], sh["lds_bytes"]) == (32, 2, True, 256, lds), sh
    obs, act = eng.trajectory_buffers(T)
    launch = eng.rollout_launcher(T, *pol, obs=obs, act=act)
    starts = _window_starts(B, B // streams, 6, 13)
    snap, gids = _timed_form_vs_oracle(oracle_lib, eng, eng.parts, obs, act, launch, cfg, pol,
                                       seed, T, L, starts, whole=True)
    assert len(gids) >= 64
    assert (snap["ep_count"][gids] >= 1).all()
    if which.startswith("c5"):
        assert snap["counters"][1][gids].sum() > 100   # the StaircaseBots went deep
    else:
        assert snap["counters"][0][gids].sum() > 0     # combats happened


@pytest.mark.parametrize("npc_policy", [1, 2])
def test_bench_moving_extras_vs_oracle(npc_policy, oracle_lib):
    """bench.py's c3_moving_npcs / c3_chasing_npcs extras as they are timed
    (rollout_rate: C3 with npc_policy RANDOM / CHASE, 65,536 games, seed 5,
    2x RandomBot, one stream, int32 rows + actions; mov_rollout_kernel), for
    3 back-to-back 128-tick launches: every game's state after each launch
    against a threaded oracle over the batch, and 8-game windows replayed
    tick by tick (every observation row and action pair) -- the reference's
    decide_npc_move override and the NPC resolution it drives
    (updater.py:116-145, 165-178)."""
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    from optimax_rogue_amd.enums import OBS_FIELDS
    cfg = EnvConfig(width=64, height=64, n_npcs=8, npc_policy=npc_policy)
    B, T, L, seed = 65536, 128, 3, 5
    eng = BatchedEngine(cfg, B, seed=seed, device=torch.device("cuda", 0))
    obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=eng.device)
    act = torch.empty((T, B, 2), dtype=torch.int8, device=eng.device)
    launch = eng.rollout_launcher(T, 1, 1, obs=obs, act=act)
    starts = _window_starts(B, B, 6, 29)
    snap, gids = _timed_form_vs_oracle(oracle_lib, eng, [eng], [obs], [act], launch, cfg, (1, 1),
                                       seed, T, L, starts, whole=True)
    assert snap["counters"][0].sum() > 0 and snap["counters"][3].sum() > 0  # combats, NPC deaths


# round 5: banks above the default 64 KiB of LDS stay paired with the tiles
# staged (the kernel's limit raised; 512-thread workgroups above half the
# LDS), and a refused raise takes the one-lane form with global tiles
BIG_BANKS = {
    # 24 x 64x64 = 96 KiB: 512 threads; RandomBots with NPCs, StaircaseBots
    "bank96_random_npcs": (dict(width=64, height=64, n_npcs=8, max_ticks=120), (1, 1), 24, None,
                           (2, 512, 98304)),
    "bank96_stairs": (dict(width=64, height=64, max_ticks=150, despawn=2), (2, 2), 24, None,
                      (2, 512, 98304)),
    # 20 x 64x64 = 80 KiB: two workgroups per CU, 256 threads
    "bank80_random": (dict(width=64, height=64, n_npcs=4, max_ticks=100), (1, 1), 20, None,
                      (2, 256, 81920)),
    # 40 x 64x64 = the whole 160 KiB
    "bank160_random": (dict(width=64, height=64, n_npcs=8, max_ticks=100), (1, 1), 40, None,
                       (2, 512, 163840)),
    # the refused raise (forced): one lane per game, tiles read from global memory
    "bank96_refused": (dict(width=64, height=64, n_npcs=8, max_ticks=100), (1, 1), 24,
                       {"ORX_REFUSE_LDS_RAISE": "1"}, (1, 256, 0)),
    # the 512-thread choice overridden: 256-thread workgroups, one per CU
    "bank96_threads256": (dict(width=64, height=64, n_npcs=8, max_ticks=100), (1, 1), 24,
                          {"ORX_ROLLOUT_THREADS": "256"}, (2, 256, 98304)),
}


@pytest.mark.parametrize("name", sorted(BIG_BANKS))
def test_big_bank_forms_vs_oracle(name, oracle_lib, monkeypatch):
    """Dungeon banks of 80-160 KiB: the launch form (lanes per game, threads
    per workgroup, LDS bytes) and 4 x 40-tick rollouts of 2,048 games against
    the oracle's literal tile model (rows, actions, state; worldgen.py:9-26,
    world.py:41-66)."""
    import torch
    from optimax_rogue_amd.enums import OBS_FIELDS
    cfg, pol, L, env, want_shape = BIG_BANKS[name]
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, v)
    lay = _bank(64, 64, L, 90 + L, (1, 2))
    B, seed, T = 2048, 91, 40
    ora = oracle_lib.Oracle(cfg, B, seed, 3, layouts=lay)
    ora.reset(episode=np.zeros(B, np.int32))
    eng = _engine(cfg, B, seed, 3, layouts=lay)
    sh = eng.rollout_shape(*pol)
    assert (sh["lanes_per_game"], sh["threads_per_block"], sh["lds_bytes"]) == want_shape, sh
    obs = torch.zeros((T, len(OBS_FIELDS), B), dtype=torch.int32, device=eng.device)
    act = torch.zeros((T, B, 2), dtype=torch.int8, device=eng.device)
    for launch in range(4):
        want_act, want_obs = _replay(ora, T, pol)
        eng.rollout(T, *pol, obs=obs, act=act)
        compare_state(eng.snapshot(), ora.export(), ora.K, f"{name} launch {launch}")
        assert np.array_equal(act.cpu().numpy(), want_act), f"{name} actions {launch}"
        assert np.array_equal(obs.cpu().numpy(), want_obs), f"{name} obs {launch}"
    s = eng.snapshot()
    assert int(s["episode"].sum()) > 0 or pol == (2, 2)
    assert s["counters"][1].sum() > 0 or pol == (1, 1)   # StaircaseBots descended
    torch.cuda.synchronize()


# bench.py's extras at their timed shapes (bench.extras: rollout_rate, seed 5,
# one BatchedEngine, 128-tick launches with both trajectory buffers): the
# form each one launches (lanes per game, nontemporal stores), and 9 launches
# = 1,152 ticks, past the max_ticks-1000 autoreset
EXTRAS_FORMS = {
    # C2: pair_rollout_kernel<0, 1, 0, false>
    "c2_4096": ("c2", 0, 4096, (1, 1), 2, False),
    # C5 at its 8-GPU share: pair_rollout_kernel<0, 2, 0, false / true>
    "c5_16384_sep_off": ("c5", 0, 16384, (2, 2), 2, False),
    "c5_16384_sep_on": ("c5", 1, 16384, (2, 2), 2, False),
    # C5 on one GPU: the one-lane rollout_kernel at 64 games per wave, nt stores
    "c5_131072_sep_off": ("c5", 0, 131072, (2, 2), 1, True),
    "c5_131072_sep_on": ("c5", 1, 131072, (2, 2), 1, True),
}


@pytest.mark.parametrize("name", sorted(EXTRAS_FORMS))
def test_bench_extras_timed_forms_vs_oracle(name, oracle_lib):
    """Each extras line of bench.py in the exact form it is timed (C2's
    4,096 games on 32x32; C5's 16,384 and 131,072 games on 128x128 with
    StaircaseBots, separation damage off -- reference semantics -- and on, at
    bench.py's sep_period 8), 9 back-to-back 128-tick launches: 64-80 sampled
    games (8-game windows, both batch ends) replayed on the oracle, every
    tick's observation row, both actions, the state after every launch
    (updater.py:76-162, staircasebot.py:9-21, randombot.py:20-21)."""
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    from optimax_rogue_amd.enums import EXT_SEPARATION_DAMAGE, OBS_FIELDS
    which, sep, B, pol, lanes, nt = EXTRAS_FORMS[name]
    cfg = getattr(EnvConfig, which)()
    if sep:
        cfg.flags, cfg.sep_period = EXT_SEPARATION_DAMAGE, 8
    T, L, seed = 128, 9, 5
    eng = BatchedEngine(cfg, B, seed=seed, device=torch.device("cuda", 0))
    shape = eng.rollout_shape(*pol)
    assert (shape["lanes_per_game"], shape["nontemporal"]) == (lanes, nt), shape
    obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=eng.device)
    act = torch.empty((T, B, 2), dtype=torch.int8, device=eng.device)
    launch = eng.rollout_launcher(T, *pol, obs=obs, act=act)
    starts = _window_starts(B, B, 6, 11)
    snap, gids = _timed_form_vs_oracle(oracle_lib, eng, [eng], [obs], [act], launch, cfg, pol,
                                       seed, T, L, starts)
    assert (snap["ep_count"][gids] >= 1).all()
    if which == "c5":   # the StaircaseBots went deep
        assert snap["counters"][1][gids].sum() > 100


def test_bad_action_and_no_autoreset():
    import torch
    cfg = dict(width=8, height=8, max_ticks=5, autoreset=0)
    eng = _engine(cfg, 256, 1)
    a = torch.full((256, 2), 5, dtype=torch.int8, device=eng.device)
    a[7, 0] = 0
    a[9, 1] = 6
    eng.step(a)
    st = eng.status.cpu().numpy()
    assert st[7] == 16 and st[9] == 16 and (np.delete(st, [7, 9]) == 1).all()
    for _ in range(10):
        eng.step(eng.policy(1, 1))
    s = eng.snapshot()
    ok = np.ones(256, bool)
    ok[[7, 9]] = False
    assert (s["tick"][ok] == 5).all() and (s["status"][ok] == 4).all()
    assert (s["tick"][~ok] == 1).all()   # stopped games stay frozen


def test_errors_raise():
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    import torch
    with pytest.raises(ValueError):
        BatchedEngine(EnvConfig(width=3), 16, device=torch.device("cuda", 0))
    eng = _engine(dict(width=8, height=8), 16, 1)
    with pytest.raises(ValueError):
        eng.step(torch.zeros((16, 2), dtype=torch.int32, device=eng.device))
    from optimax_rogue_amd._lib import OrxError
    with pytest.raises(OrxError):
        eng.rollout(4, 0, 1)


def test_empty_batch():
    eng = _engine(dict(width=8, height=8), 0, 1)
    eng.step(eng.policy(1, 1))
    eng.rollout(3, 1, 1)


def _kat_cases():
    from golden_util import Kat
    k = Kat()
    return [k.case(i) for i in range(len(k.names))]


@pytest.mark.parametrize("case", _kat_cases(), ids=lambda c: c["name"])
def test_known_answer_scenarios(case):
    """SURVEY.md s4's semantics probes through orx_step_events and orx_step:
    the hand-built state loaded into the engine, one tick, events and state
    equal to the reference's (tests/golden/kat_scenarios.npz)."""
    import torch
    from golden_util import Kat
    cfg = Kat().cfg
    K = cfg["n_npcs"]
    for events in (True, False):
        eng = _engine(cfg, 1, case["seed"])
        snap = eng.snapshot()
        npc_pos = np.full((K, 1), 0xFFFF, np.int64)
        npc_hp = np.zeros((K, 1), np.int64)
        alive = 0
        for iden, d, x, y, hp in case["ents"]:
            if iden <= 2:
                for f, v in (("p_x", x), ("p_y", y), ("p_depth", d), ("p_health", hp)):
                    snap[f][iden - 1][0] = v
            else:
                npc_pos[iden - 3, 0] = x | (y << 8)
                npc_hp[iden - 3, 0] = hp
                alive |= 1 << (iden - 3)
        snap.update(st_x=np.full((2, 1), 5), st_y=np.full((2, 1), 5), tick=np.array([1]),
                    status=np.array([1]), episode=np.array([0]), npc_pos=npc_pos,
                    npc_health=npc_hp, npc_alive=np.array([alive]))
        eng.load_snapshot(snap)
        acts = torch.tensor([case["moves"]], dtype=torch.int8, device=eng.device)
        if events:
            _, ev, n = eng.step(acts, events=True)
            ev, n = ev.cpu().numpy(), int(n.cpu().numpy()[0])
            assert [tuple(int(v) for v in r) for r in ev[0, :n]] == case["events"], case["name"]
        else:
            eng.step(acts)
        s = eng.snapshot()
        for k, v in case["final"].items():
            got = np.asarray(s[k])
            got = got[:, 0] if got.ndim == 2 else got[:1]
            want = np.asarray(v).reshape(-1)[: got.size].reshape(got.shape)
            if k == "npc_health":   # dead slots keep their last value; compare live ones
                live = [j for j in range(K) if (int(case["final"]["npc_alive"]) >> j) & 1]
                got, want = got[live], want[live]
            assert np.array_equal(got, want), (case["name"], events, k, got, want)
        torch.cuda.synchronize()


# The paired rollout form (pair_rollout_kernel: two lanes per game, one per
# player) on its own: NPC-free StaircaseBot pairs with and without separation
# damage, Together and Separated starts, both despawn rules, short episodes
# (the paired reset and descend fast paths and their general fallbacks), and
# RandomBot pairs with register NPCs -- trajectories and state against the
# oracle's policy + step, tick by tick.
PAIRED_CASES = {
    "stairs_sep_damage": (dict(width=12, height=10, start_mode=2, p1_depth=0, p2_depth=2,
                               max_ticks=60, flags=1, sep_period=2), (2, 2), 1000, 61),
    "stairs_sep_damage_unused": (dict(width=9, height=14, despawn=2, max_ticks=40, flags=1,
                                      sep_period=3, player_health=4), (2, 2), 777, 62),
    "stairs_sep_period1_frail": (dict(width=7, height=7, start_mode=2, p1_depth=1, p2_depth=0,
                                      max_ticks=0, flags=1, sep_period=1, player_health=3),
                                 (2, 2), 1531, 63),
    "stairs_short_episodes": (dict(width=20, height=20, max_ticks=25), (2, 2), 1531, 64),
    "stairs_separated_64": (dict(width=64, height=64, start_mode=2, p1_depth=3, p2_depth=1,
                                 max_ticks=90, despawn=2), (2, 2), 2048, 65),
    "random_npcs_resets": (dict(width=10, height=10, n_npcs=5, max_ticks=30), (1, 1), 1000, 66),
    "random_duel_deaths": (dict(width=4, height=5, max_ticks=0, player_health=2), (1, 1), 500,
                           67),
    # the 16-slot register-NPC instances (K 9..16) with RandomBots
    "random_npcs_k12": (dict(width=9, height=8, n_npcs=12, npc_health=2, max_ticks=45), (1, 1),
                        1000, 68),
    "random_npcs_k16_unused": (dict(width=10, height=9, n_npcs=16, max_ticks=35, despawn=2),
                               (1, 1), 999, 69),
    # StaircaseBots with register NPCs (rare_tick's general path in the pair):
    # player 2 starts above the NPCs' depth and descends onto it, where
    # player 1 walks through them
    "stairs_npcs_separated": (dict(width=8, height=7, n_npcs=6, start_mode=2, p1_depth=1,
                                   p2_depth=0, max_ticks=50, npc_health=2), (2, 2), 1000, 70),
    "stairs_npcs_k14_unused": (dict(width=9, height=9, n_npcs=14, start_mode=2, p1_depth=1,
                                    p2_depth=0, despawn=2, max_ticks=40), (2, 2), 1024, 71),
    # separation damage's multiply-shift ceil(k / period) (round 5) over long
    # separations and at the largest period ORX_SEP_PERIOD_MAX
    "stairs_sep_period7_long": (dict(width=16, height=16, start_mode=2, p1_depth=0, p2_depth=3,
                                     max_ticks=0, flags=1, sep_period=7, player_health=40),
                                (2, 2), 1000, 76),
    "stairs_sep_period_max": (dict(width=12, height=12, start_mode=2, p1_depth=0, p2_depth=2,
                                   max_ticks=70, flags=1, sep_period=1 << 24, player_health=3),
                              (2, 2), 777, 77),
}


# round 4: the paired form with the character mechanics (PM 3: mana,
# experience, items; parity unpinned vs the reference, engine vs oracle) and
# with a dungeon bank (walls, several staircases per layout; PM 1 with NPCs,
# PM 2 under both despawn rules, PM 3)
PAIRED_CASES.update({
    "rpg_npcs": (dict(width=10, height=9, n_npcs=8, npc_health=2, max_ticks=45,
                      flags=4 | 16 | 32, xp_per_level=2, item_drop_pct=70), (1, 1), 1000, 72),
    "rpg_heal_flag_k14": (dict(width=9, height=9, n_npcs=14, max_ticks=40, flags=4 | 8 | 16 | 32,
                               mana_max=12, item_bonus=2), (1, 1), 1024, 73),
    "bank_random_npcs": (dict(width=20, height=16, n_npcs=8, max_ticks=50), (1, 1), 1000, 74),
    "bank_stairs_unused": (dict(width=12, height=10, max_ticks=60, despawn=2, start_mode=2,
                                p1_depth=2, p2_depth=0), (2, 2), 1000, 75),
    "bank_stairs_npcs": (dict(width=14, height=12, n_npcs=5, max_ticks=60), (2, 2), 1001, 76),
    "bank_rpg": (dict(width=16, height=12, n_npcs=8, npc_health=2, max_ticks=50,
                      flags=4 | 16 | 32, item_drop_pct=60), (1, 1), 1000, 77),
})
# round 4: the StaircaseBot form's lean spans (greedy walks with no staircase
# target, meet or episode end ahead) on grids large enough that whole waves
# walk lean for many ticks: episodes ending inside a span, separation damage
# (lean only while the depths agree), players on different depths
PAIRED_CASES.update({
    "stairs_lean_spans": (dict(width=96, height=96, max_ticks=150), (2, 2), 256, 85),
    "stairs_lean_sep": (dict(width=96, height=96, max_ticks=120, flags=1, sep_period=4), (2, 2),
                        256, 86),
    "stairs_lean_separated": (dict(width=80, height=80, start_mode=2, p1_depth=0, p2_depth=1,
                                   max_ticks=130), (2, 2), 256, 87),
})
# round 5: a RandomBot against a StaircaseBot (PM 4: player 1 random, PM 5:
# player 2), NPC-free and with register NPCs, both starts and despawn rules,
# short episodes (the reset and descend fast paths, the lean meet, NPC hits)
PAIRED_CASES.update({
    "mixed_rs_npcs": (dict(width=10, height=10, n_npcs=6, max_ticks=40), (1, 2), 1000, 91),
    "mixed_sr_npcs16_unused": (dict(width=9, height=9, n_npcs=14, max_ticks=35, despawn=2),
                               (2, 1), 1000, 92),
    "mixed_rs_separated": (dict(width=12, height=10, start_mode=2, p1_depth=1, p2_depth=0,
                                max_ticks=60), (1, 2), 1000, 93),
    "mixed_sr_duel": (dict(width=5, height=4, max_ticks=30, player_health=3), (2, 1), 1000, 94),
    "mixed_rs_c3_shape": (dict(width=64, height=64, n_npcs=8, max_ticks=80), (1, 2), 1024, 95),
    # StaircaseBots hitting NPCs on the paired NPC-hit path, with separation damage
    "stairs_sep_npcs": (dict(width=10, height=9, start_mode=2, p1_depth=0, p2_depth=1, n_npcs=5,
                             max_ticks=50, flags=1, sep_period=3), (2, 2), 1000, 96),
})
PAIRED_BANKS = {"bank_random_npcs": (20, 16, 6, 81, (1, 2)), "bank_stairs_unused": (12, 10, 5, 82, (1, 2)),
                "bank_stairs_npcs": (14, 12, 4, 83, (2,)), "bank_rpg": (16, 12, 5, 84, (1, 3))}


@pytest.mark.parametrize("name", sorted(PAIRED_CASES))
def test_paired_rollout_vs_oracle(name, oracle_lib):
    import torch
    from optimax_rogue_amd.enums import OBS_FIELDS
    cfg, pol, B, seed = PAIRED_CASES[name]
    lay = _bank(*PAIRED_BANKS[name]) if name in PAIRED_BANKS else None
    ora = oracle_lib.Oracle(cfg, B, seed, 5, layouts=lay)
    ora.reset(episode=np.zeros(B, np.int32))
    eng = _engine(cfg, B, seed, 5, layouts=lay)
    assert eng.rollout_shape(*pol)["lanes_per_game"] == 2, name
    T = 40
    obs = torch.zeros((T, len(OBS_FIELDS), B), dtype=torch.int32, device=eng.device)
    act = torch.zeros((T, B, 2), dtype=torch.int8, device=eng.device)
    episodes = 0
    for launch in range(4):
        want_act, want_obs = _replay(ora, T, pol)
        eng.rollout(T, *pol, obs=obs, act=act)
        compare_state(eng.snapshot(), ora.export(), ora.K, f"{name} launch {launch}")
        assert np.array_equal(act.cpu().numpy(), want_act), f"{name} actions {launch}"
        assert np.array_equal(obs.cpu().numpy(), want_obs), f"{name} obs {launch}"
    episodes = int(eng.snapshot()["episode"].sum())
    assert episodes > 0, name   # every case crosses resets
    if cfg.get("n_npcs"):
        c = eng.snapshot()["counters"]
        assert c[0].sum() > 0 and c[3].sum() > 0, name   # combats and NPC deaths happened
    torch.cuda.synchronize()


@pytest.mark.parametrize("wh", [(300, 260), (256, 256)])
def test_wide_grid_rollout_form_vs_oracle(wh, oracle_lib):
    """The paired form packs cells as x | y << 8, so it runs only on grids up
    to 256 x 256; a wider NPC-free grid takes the one-lane form (round 3's
    plan paired it and would have rebuilt x from 8 bits).  StaircaseBots
    (they reach the far cells) against the oracle."""
    import torch
    from optimax_rogue_amd.enums import OBS_FIELDS
    W, H = wh
    cfg = dict(width=W, height=H, max_ticks=400)
    B, T, seed = 512, 150, 31
    ora = oracle_lib.Oracle(cfg, B, seed, 0)
    ora.reset(episode=np.zeros(B, np.int32))
    eng = _engine(cfg, B, seed)
    assert eng.rollout_shape(2, 2)["lanes_per_game"] == (2 if W <= 256 else 1)
    obs = torch.zeros((T, len(OBS_FIELDS), B), dtype=torch.int32, device=eng.device)
    act = torch.zeros((T, B, 2), dtype=torch.int8, device=eng.device)
    for launch in range(3):
        want_act, want_obs = _replay(ora, T, (2, 2))
        eng.rollout(T, 2, 2, obs=obs, act=act)
        compare_state(eng.snapshot(), ora.export(), 0, f"{wh} launch {launch}")
        assert np.array_equal(act.cpu().numpy(), want_act), f"{wh} actions {launch}"
        assert np.array_equal(obs.cpu().numpy(), want_obs), f"{wh} obs {launch}"
    assert (eng.snapshot()["p_x"] > 255).any() or W <= 256


def test_dense_npc_character_trajectory_vs_oracle(oracle_lib):
    """Dense NPCs (K > 16) with the character mechanics and RandomBots, WITH
    trajectory buffers: the generic rollout form (there is no dense instance
    of the PM 3 form; before round 4 this launch matched no kernel and
    returned without running) -- rows, actions and state vs the oracle."""
    import torch
    from optimax_rogue_amd.enums import OBS_FIELDS
    cfg = dict(width=12, height=12, n_npcs=30, npc_health=2, max_ticks=60, flags=4 | 16 | 64,
               xp_per_level=2)
    B, T, seed = 1024, 30, 45
    ora = oracle_lib.Oracle(cfg, B, seed, 0)
    ora.reset(episode=np.zeros(B, np.int32))
    eng = _engine(cfg, B, seed)
    obs = torch.zeros((T, len(OBS_FIELDS), B), dtype=torch.int32, device=eng.device)
    act = torch.zeros((T, B, 2), dtype=torch.int8, device=eng.device)
    for launch in range(3):
        want_act, want_obs = _replay(ora, T, (1, 1))
        eng.rollout(T, 1, 1, obs=obs, act=act)
        compare_state(eng.snapshot(), ora.export(), ora.K, f"launch {launch}")
        assert np.array_equal(act.cpu().numpy(), want_act), f"actions {launch}"
        assert np.array_equal(obs.cpu().numpy(), want_obs), f"obs {launch}"
    assert int(eng.snapshot()["episode"].sum()) > 0


# ORX_OBS_COMPACT trajectory rows: every launch form -- the paired compact
# instances (the bench's C3 shards, C2, C5 with separation damage), the
# one-lane compact instances (C5 and C3 at full waves), and the generic form
# that reads the format at run time (character mechanics, a dungeon bank,
# dense NPCs, stock seeding) -- decodes to exactly the int32 rows of the same
# launches, with identical actions and state.
COMPACT_FORMS = {
    "c3_bench_shards": (dict(width=64, height=64, n_npcs=8), (1, 1), 65536, 2, 2),
    "c2_pair": (dict(width=32, height=32, max_ticks=90), (1, 1), 4096, 1, 2),
    "c5_pair_sep": (dict(width=128, height=128, flags=1, sep_period=8), (2, 2), 16384, 1, 2),
    "c5_one_lane": (dict(width=128, height=128), (2, 2), 131072, 1, 1),
    "c3_one_lane": (dict(width=64, height=64, n_npcs=8, max_ticks=90), (1, 1), 65536, 1, 1),
    # int32 rows: the paired character form; compact rows: the generic form
    "rpg_pair_vs_generic": (dict(width=16, height=16, n_npcs=8, flags=4 | 16 | 32, max_ticks=80),
                            (1, 1), 4096, 1, 2),
    "bank_generic": (dict(width=20, height=16, n_npcs=4, max_ticks=70), (2, 1), 3001, 1, 1),
    "dense_generic": (dict(width=12, height=12, n_npcs=30, max_ticks=60), (1, 2), 2048, 1, 1),
    "stock_mt": (dict(width=10, height=9, n_npcs=4, max_ticks=60, rng=1), (1, 2), 1024, 1, 1),
}


@pytest.mark.parametrize("name", sorted(COMPACT_FORMS))
def test_compact_rows_vs_oracle(name, oracle_lib):
    """Round 5: every compact-row launch form against the oracle first hand
    (not only against the engine's own int32 rows): 3 launches, sampled
    8-game windows (both ends of each shard) replayed tick by tick -- the
    decoded rows, both actions and the state after each launch."""
    import torch
    from optimax_rogue_amd import DungeonBank, EnvConfig
    from optimax_rogue_amd.engine import StreamShardedEngine
    from optimax_rogue_amd.enums import OBS_COMPACT
    cfgd, pol, B, streams, lanes = COMPACT_FORMS[name]
    layouts = DungeonBank.random(20, 16, 6, seed=3, n_stairs=2).layouts \
        if name == "bank_generic" else None
    cfg = EnvConfig.from_dict(cfgd, layouts=layouts)
    T, L, seed, off = (64 if B >= 65536 else 100), 3, 21, 3
    eng = StreamShardedEngine(cfg, B, seed=seed, game_offset=off, device=torch.device("cuda", 0),
                              n_streams=streams)
    if name != "stock_mt":
        assert eng.rollout_shape(*pol)["lanes_per_game"] == lanes, name
    obs, act = eng.trajectory_buffers(T, OBS_COMPACT)
    launch = eng.rollout_launcher(T, *pol, obs=obs, act=act, obs_format=OBS_COMPACT)
    starts = _window_starts(B - B % 8, max(8, (B // streams) // 8 * 8), 4, 29)
    _timed_form_vs_oracle(oracle_lib, eng, eng.parts, obs, act, launch, cfg, pol, seed, T, L,
                          starts, off, compact=True)


@pytest.mark.parametrize("name", sorted(COMPACT_FORMS))
def test_compact_rows_equal_int32_rows(name):
    import torch
    from optimax_rogue_amd import DungeonBank, EnvConfig
    from optimax_rogue_amd.engine import StreamShardedEngine, decode_compact
    from optimax_rogue_amd.enums import OBS_COMPACT, OBS_INT32
    cfgd, pol, B, streams, lanes = COMPACT_FORMS[name]
    layouts = DungeonBank.random(20, 16, 6, seed=3, n_stairs=2).layouts \
        if name == "bank_generic" else None
    cfg = EnvConfig.from_dict(cfgd, layouts=layouts)
    dev = torch.device("cuda", 0)
    T = 64 if B >= 65536 else 100
    res = []
    for fmt in (OBS_INT32, OBS_COMPACT):
        eng = StreamShardedEngine(cfg, B, seed=21, game_offset=3, device=dev, n_streams=streams)
        if name != "stock_mt" and fmt == OBS_INT32:
            assert eng.rollout_shape(*pol)["lanes_per_game"] == lanes, name
        obs, act = eng.trajectory_buffers(T, fmt)
        go = eng.rollout_launcher(T, *pol, obs=obs, act=act, obs_format=fmt)
        rows, acts = [], []
        for _ in range(2):
            eng.fork()
            go()
            eng.join()
            o = torch.cat(obs, dim=2)
            rows.append((decode_compact(o) if fmt == OBS_COMPACT else o).cpu().numpy())
            acts.append(torch.cat(act, dim=1).cpu().numpy())
        res.append((rows, acts, eng.snapshot()))
        del eng, obs, act
        torch.cuda.empty_cache()
    (r0, a0, s0), (r1, a1, s1) = res
    for k in range(2):
        assert np.array_equal(r0[k], r1[k]), (name, k)
        assert np.array_equal(a0[k], a1[k]), (name, k)
    for k in s0:
        assert np.array_equal(s0[k], s1[k]), (name, k)
    assert s0["ep_count"].sum() > 0 or name.startswith("c3_bench") or name.startswith("c5")


@pytest.mark.parametrize("name", case_names())
def test_golden_step_n(name):
    """orx_step_n: a fixture's whole recorded move log in one launch -- every
    tick's observation row and the final state equal the reference's
    (server/main.py:110-113 over updater.py:76-162).  Keyed-stream fixtures
    only: in stock-seed mode the bots' draws share the game's stream, which a
    replay of given moves does not draw (orx_step_n refuses that mode)."""
    import torch
    from optimax_rogue_amd.enums import OBS_FIELDS
    fx = Fixture(name)
    if fx.stock:
        pytest.skip("stock-seed fixture: replayed tick by tick (test_golden_step_given_actions)")
    eng = _engine(fx.cfg, fx.G, fx.seed, fx.game_offset, layouts=fx.layouts)
    acts = torch.from_numpy(np.ascontiguousarray(fx.actions)).to(eng.device)
    obs = torch.zeros((fx.T, len(OBS_FIELDS), fx.G), dtype=torch.int32, device=eng.device)
    eng.step_n(acts, obs=obs)
    o = obs.cpu().numpy()
    for t in range(fx.T):
        assert np.array_equal(o[t], _obs_rows(fx.state(t + 1))), f"{name} obs t={t + 1}"
    compare_state(eng.snapshot(), fx.state(fx.T), fx.K, f"{name} final")


def test_replay_bench_shape_fast_equals_generic():
    """bench.py's replay_step_n extra in the form it is timed (C3, 65,536
    games, a 128-tick uniform move log, int32 rows: the fast replay_kernel at
    64 games per wave) equals the generic one-lane form (ORX_STEP_N_GENERIC=1,
    itself checked tick by tick against orx_step and the reference fixtures):
    every row and the final state, over two consecutive logs."""
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    from optimax_rogue_amd.enums import OBS_FIELDS
    dev = torch.device("cuda", 0)
    B, T = 65536, 128
    g = torch.Generator(device="cpu").manual_seed(11)
    logs = [torch.randint(1, 6, (T, B, 2), generator=g, dtype=torch.int8).to(dev)
            for _ in range(2)]
    res = []
    for generic in ("0", "1"):
        os.environ["ORX_STEP_N_GENERIC"] = generic
        try:
            eng = BatchedEngine(EnvConfig.c3(), B, seed=3, device=dev)
            rows = []
            for log in logs:
                obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
                eng.step_n(log, obs=obs)
                rows.append(obs.cpu().numpy())
            torch.cuda.synchronize()
        finally:
            del os.environ["ORX_STEP_N_GENERIC"]
        res.append((rows, eng.snapshot()))
    (r0, s0), (r1, s1) = res
    for k in range(2):
        assert np.array_equal(r0[k], r1[k]), k
    for k in s0:
        assert np.array_equal(s0[k], s1[k]), k
    assert s0["ep_count"].sum() > 0 and s0["counters"][0].sum() > 0


@pytest.mark.parametrize("paired", ["plan", "1", "0", "shards"])
def test_replay_bench_shape_vs_oracle(paired, oracle_lib, monkeypatch):
    """bench.py's replay_step_n extra as it is timed (C3, 65,536 games, seed
    3, 128-tick uniform move logs, int32 rows: the fast replay_kernel) against
    the C oracle over every game (a threaded pool stepping the same logs):
    every tick's 14-field row of all 65,536 games and the final state, over
    two consecutive logs (server/main.py:110-113 over updater.py:76-162);
    in the form the plan picks and with the paired LOG form forced on / off
    (ORX_REPLAY_PAIRED); and as two stream shards
    (StreamShardedEngine.replay_launcher, "shards")."""
    import torch
    from oracle_pool import OraclePool
    if paired not in ("plan", "shards"):
        monkeypatch.setenv("ORX_REPLAY_PAIRED", paired)
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine, StreamShardedEngine
    from optimax_rogue_amd.enums import OBS_FIELDS
    dev = torch.device("cuda", 0)
    B, T, seed = 65536, 128, 3
    cfg = EnvConfig.c3()
    if paired == "shards":
        eng = StreamShardedEngine(cfg, B, seed=seed, device=dev, n_streams=2)
    else:
        eng = BatchedEngine(cfg, B, seed=seed, device=dev)
    pool = OraclePool(oracle_lib, cfg.to_dict(), B, seed)
    g = torch.Generator(device="cpu").manual_seed(11)
    for k in range(2):
        log = torch.randint(1, 6, (T, B, 2), generator=g, dtype=torch.int8)
        if paired == "shards":
            obs_l, _ = eng.trajectory_buffers(T)
            eng.fork()
            eng.replay_launcher(eng.split_log(log.to(dev)), obs_l)()
            eng.join()
            rows = torch.cat(obs_l, dim=2).cpu().numpy()
        else:
            obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
            eng.step_n(log.to(dev), obs=obs)
            rows = obs.cpu().numpy()
        ln = log.numpy()
        for t in range(T):
            pool.step(ln[t])
            assert np.array_equal(rows[t], _obs_rows(pool.export())), (k, t)
    s = eng.snapshot()
    compare_state(s, pool.export(), cfg.n_npcs, "replay final")
    assert s["counters"][0].sum() > 0 and s["counters"][3].sum() > 0


def test_vecenv_bench_shape_vs_oracle(oracle_lib):
    """VecEnv.step at bench.py's vecenv_step shape (C3, 65,536 games, int64
    learner actions for player 1, a RandomBot opponent) against the C oracle
    over every game: the action pair played, the observation row, reward,
    done and status of all 65,536 games every tick (optimax_rogue_bots/
    main.py:118-155, randombot.py:20-21, updater.py:76-162)."""
    import torch
    from oracle_pool import OraclePool
    from optimax_rogue_amd import EnvConfig, VecEnv
    dev = torch.device("cuda", 0)
    B, T, seed = 65536, 40, 3
    cfg = EnvConfig.c3()
    cfg.max_ticks = 25          # episodes end (reward / done) inside the window
    env = VecEnv(cfg, B, seed=seed, device=dev, opponent=1, out_buffers=2)
    pool = OraclePool(oracle_lib, cfg.to_dict(), B, seed)
    g = torch.Generator(device="cpu").manual_seed(17)
    before = pool.export()["status"]
    dones = 0
    for t in range(T):
        a = torch.randint(1, 6, (B,), generator=g, dtype=torch.int64)
        obs, r, d, st = (x.cpu().numpy() for x in env.step(a.to(dev)))
        acts = np.full((B, 2), 5, np.int8)
        acts[:, 0] = a.numpy()
        acts = pool.policy(0, 1, acts)       # player 2's RandomBot
        pool.step(acts)
        want = pool.export()
        assert np.array_equal(env.engine.actions.cpu().numpy(), acts), t
        assert np.array_equal(obs, _obs_rows(want).T), t
        assert np.array_equal(st, want["status"]), t
        ended = (before == 1) & (want["status"] >= 2) & (want["status"] <= 4)
        assert np.array_equal(d, ended), t
        assert np.array_equal(r, np.where(ended, (want["status"] == 2).astype(np.float32)
                                          - (want["status"] == 3), 0).astype(np.float32)), t
        before = want["status"]
        dones += int(d.sum())
    compare_state(env.engine.snapshot(), pool.export(), cfg.n_npcs, "vecenv final")
    assert dones >= B


STEP_N_CASES = {
    "npc8": (dict(width=16, height=16, n_npcs=8, max_ticks=90), None),
    "dense30": (dict(width=12, height=12, n_npcs=30, npc_health=2, max_ticks=70), None),
    "bank_unused": (dict(width=12, height=10, n_npcs=3, max_ticks=60, despawn=2, start_mode=2,
                         p1_depth=1, p2_depth=0), (12, 10, 5, 88, (1, 2))),
    "rpg_readme": (dict(width=9, height=9, n_npcs=6, max_ticks=60, flags=4 | 8 | 16 | 32 | 64,
                        player_health=6), None),
    "sep_double": (dict(width=7, height=7, start_mode=2, p1_depth=0, p2_depth=1, max_ticks=0,
                        flags=3, sep_period=2, player_health=4), None),
    "c3": (dict(width=64, height=64, n_npcs=8, max_ticks=1000), None),
    "npc16_unused": (dict(width=20, height=14, n_npcs=16, npc_health=1, despawn=2, start_mode=2,
                          p1_depth=0, p2_depth=2, max_ticks=120), None),
    "heal_mana": (dict(width=8, height=8, n_npcs=4, max_ticks=50, flags=4 | 8,
                       player_health=5), None),
    "no_autoreset": (dict(width=6, height=6, n_npcs=2, max_ticks=40, autoreset=0), None),
}


@pytest.mark.parametrize("name", sorted(STEP_N_CASES))
def test_step_n_equals_step(name):
    """orx_step_n over 160 ticks of random moves (~1% of them invalid: the
    game stops with STATUS_BAD_ACTION and restarts) equals 160 orx_step calls:
    the state after every tick (its observation row) and at the end; the
    compact rows decode to the same rows, and a launch without rows ends in
    the same state.  Register NPCs on empty dungeons take the fast form
    (replay_kernel: the rollout's tick on the logged pairs), dense NPCs and
    banks the generic one; ORX_STEP_N_GENERIC=1 forces the generic form on
    the fast form's cases, with the same result."""
    import torch
    from optimax_rogue_amd.engine import decode_compact
    from optimax_rogue_amd.enums import EXT_HEAL, OBS_COMPACT, OBS_FIELDS
    cfg, bank = STEP_N_CASES[name]
    lay = _bank(*bank) if bank else None
    B, T, seed = 1500, 160, 7
    hi = 6 if cfg.get("flags", 0) & EXT_HEAL else 5
    rs = np.random.RandomState(3)
    acts = rs.randint(1, hi + 1, size=(T, B, 2)).astype(np.int8)
    bad = rs.rand(T, B, 2) < 0.005
    acts[bad] = rs.choice([0, -3, hi + 1, 100], size=int(bad.sum())).astype(np.int8)
    a = torch.from_numpy(acts).to("cuda:0")
    ref = _engine(cfg, B, seed, 11, layouts=lay)
    eng = _engine(cfg, B, seed, 11, layouts=lay)
    obs = torch.zeros((T, len(OBS_FIELDS), B), dtype=torch.int32, device=eng.device)
    eng.step_n(a, obs=obs)
    o = obs.cpu().numpy()
    stops = 0
    for t in range(T):
        st = ref.step(a[t].contiguous())
        snap = ref.snapshot()
        assert np.array_equal(o[t], _obs_rows(snap)), f"{name} t={t}"
        stops += int((snap["status"] == 16).sum())
    compare_state(eng.snapshot(), ref.snapshot(), int(cfg.get("n_npcs", 0)), f"{name} final")
    assert stops > 0
    eng3 = _engine(cfg, B, seed, 11, layouts=lay)
    eng3.step_n(a)
    compare_state(eng3.snapshot(), ref.snapshot(), int(cfg.get("n_npcs", 0)), f"{name} no rows")
    if bank is None and int(cfg.get("n_npcs", 0)) <= 16:
        os.environ["ORX_STEP_N_GENERIC"] = "1"
        try:
            eng4 = _engine(cfg, B, seed, 11, layouts=lay)
            g_obs = torch.zeros_like(obs)
            eng4.step_n(a, obs=g_obs)
            torch.cuda.synchronize()
        finally:
            del os.environ["ORX_STEP_N_GENERIC"]
        assert np.array_equal(g_obs.cpu().numpy(), o), f"{name} generic form"
        # the paired LOG form (pair_rollout_kernel PM 6, the plan's choice at
        # this batch when the flags are 0) against the one-lane replay_kernel
        for form in ("0", "1"):
            os.environ["ORX_REPLAY_PAIRED"] = form
            try:
                eng5 = _engine(cfg, B, seed, 11, layouts=lay)
                p_obs = torch.zeros_like(obs)
                eng5.step_n(a, obs=p_obs)
                torch.cuda.synchronize()
            finally:
                del os.environ["ORX_REPLAY_PAIRED"]
            assert np.array_equal(p_obs.cpu().numpy(), o), f"{name} ORX_REPLAY_PAIRED={form}"
            compare_state(eng5.snapshot(), ref.snapshot(), int(cfg.get("n_npcs", 0)),
                          f"{name} ORX_REPLAY_PAIRED={form} final")
    if int(cfg.get("max_ticks", 0)) > 0 and not cfg.get("flags", 0) & 1:
        eng2 = _engine(cfg, B, seed, 11, layouts=lay)
        c_obs = torch.zeros((T, 6, B), dtype=torch.int32, device=eng.device)
        eng2.step_n(a, obs=c_obs, obs_format=OBS_COMPACT)
        assert np.array_equal(decode_compact(c_obs).cpu().numpy(), o), name
