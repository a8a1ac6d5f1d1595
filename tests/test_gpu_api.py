"""GPU: the host-side mirror of the reference interface (BatchedUpdater,
compat views, BotDriver) on the HIP engine."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class ToStairsBot:
    """A Bot (optimax_rogue_bots/bot.py interface) that walks to the staircase
    of its view, horizontal axis first when strictly farther."""

    def __init__(self, iden):
        self.iden = iden
        self.finished_with = None

    def started(self, gs):
        pass

    def on_move(self, gs, mv):
        pass

    def finished(self, gs, result):
        self.finished_with = int(result)

    def move(self, gs):
        me = gs.iden_lookup[self.iden]
        sx, sy = gs.world.dungeons[me.depth].staircase()
        dx, dy = sx - me.x, sy - me.y
        if abs(dx) > abs(dy):
            return 2 if dx > 0 else 4
        return 3 if dy > 0 else 1


def test_batched_updater_matches_oracle(oracle_lib):
    import torch
    from optimax_rogue_amd import DungeonDespawningStrategy
    from optimax_rogue_amd.updater import BatchedUpdater
    B = 512
    upd = BatchedUpdater((9, 9), DungeonDespawningStrategy.Unused, 60, n_games=B, seed=5,
                         n_npcs=2, device=torch.device("cuda", 0))
    o = oracle_lib.Oracle(upd.engine.cfg.to_dict(), B, 5)
    o.reset()
    rng = np.random.default_rng(1)
    for t in range(100):
        a = rng.integers(1, 6, size=(B, 2)).astype(np.int8)
        res = upd.update(a[:, 0], a[:, 1]).cpu().numpy()
        o.step(a)
        assert np.array_equal(res, o.export()["status"]), t
    gs = upd.game_state(3)
    assert gs.tick == int(o.export()["tick"][3])


def test_bot_driver(oracle_lib):
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.compat import BotDriver
    from optimax_rogue_amd.engine import BatchedEngine
    B = 64
    cfg = EnvConfig(width=8, height=8, max_ticks=30, autoreset=0)
    eng = BatchedEngine(cfg, B, seed=2, device=torch.device("cuda", 0))
    ref = BatchedEngine(cfg, B, seed=2, device=torch.device("cuda", 0))
    bots = [[ToStairsBot(1 + p) for _ in range(B)] for p in range(2)]
    drv = BotDriver(eng, bots[0], bots[1])
    for t in range(35):
        drv.step()
        ref.step(ref.policy(2, 2))
        s1, s2 = eng.snapshot(), ref.snapshot()
        for k in ("p_x", "p_y", "p_depth", "tick", "status"):
            assert np.array_equal(s1[k], s2[k]), (t, k)
    assert all(b.finished_with in (2, 3, 4) for b in bots[0])   # every game ended


@pytest.mark.parametrize("name", __import__("golden_util").case_names())
def test_engine_game_states_codec(name, oracle_lib):
    """Engine state -> full reference-schema GameState (World.dungeons
    regenerated on the GPU) -> serializer bytes equal to the reference's for
    Together/Unreachable games; GameState.__eq__-equal (dict order ignored)
    for the others."""
    import torch
    from golden_util import Fixture
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    from test_compat import oracle_view
    fx = Fixture(name)
    cfg = EnvConfig.from_dict(fx.cfg, layouts=fx.layouts)
    eng = BatchedEngine(cfg, fx.G, seed=fx.seed, game_offset=fx.game_offset,
                        device=torch.device("cuda", 0))
    o = oracle_lib.Oracle(fx.cfg, fx.G, fx.seed, fx.game_offset, layouts=fx.layouts)
    o.reset(episode=np.zeros(fx.G, np.int32))
    exact = cfg.start_mode == 1 and cfg.despawn == 1
    ticks = set(int(t) for t in fx.z["ser_ticks"])
    acts = torch.from_numpy(fx.actions).to(eng.device)
    for t in range(fx.T + 1):
        if t in ticks:
            views = eng.game_states()
            for g in range(fx.G):
                if exact:
                    assert views[g].serialize() == fx.serialized(t, g), (name, t, g)
                else:
                    assert views[g] == oracle_view(o, g, cfg), (name, t, g)
        if t < fx.T:
            if fx.stock:   # the bots' draws share each game's random stream
                eng.policy(*fx.policy)
                o.policy(*fx.policy)
            eng.step(acts[t].contiguous())
            o.step(fx.actions[t])


def _as_record(u):
    from optimax_rogue_amd import updates as U
    if isinstance(u, U.EntityCombatUpdate):
        (flag,) = tuple(u.tags)
        return (1, u.attacker_iden, u.defender_iden, int(flag))
    if isinstance(u, U.EntityDeathUpdate):
        return (2, u.entity_iden, 0, 0)
    if isinstance(u, U.EntityPositionUpdate):
        return (3, u.entity_iden, u.depth, (u.posx & 0xFFFF) | (u.posy << 16))
    return (4, 0, u.depth, 0)


@pytest.mark.parametrize("name,g", [("small_npc_random", 0), ("small_npc_random", 5),
                                    ("stairs_unreachable", 2), ("duel_5", 1),
                                    ("separated_unused", 3), ("bank_random_npc", 4),
                                    ("bank_stairs_unused", 1)])
def test_game_updater_drop_in(name, g):
    """GameUpdater.update(gs, m1, m2) -> (UpdateResult, updates) over one
    fixture game: the returned updates equal the reference's, applying them
    keeps the caller's GameState equal to the engine's, and the results match."""
    import torch
    from golden_util import Fixture
    from optimax_rogue_amd import DungeonDespawningStrategy, UpdateResult
    from optimax_rogue_amd.updater import GameUpdater
    from optimax_rogue_amd import DungeonBank
    fx = Fixture(name)
    c = fx.cfg
    start = "together" if c["start_mode"] == 1 else ("separated", c["p1_depth"], c["p2_depth"])
    dgen = (c["width"], c["height"]) if fx.layouts is None else DungeonBank(fx.layouts)
    upd = GameUpdater(dgen, DungeonDespawningStrategy(c["despawn"]),
                      c["max_ticks"] or None, seed=fx.seed, game_id=fx.game_offset + g,
                      game_start=start, n_npcs=c["n_npcs"], device=torch.device("cuda", 0))
    gs = upd.setup_game()
    s0 = fx.state(0)
    assert (gs.player_1.x, gs.player_1.y) == (s0["p_x"][0][g], s0["p_y"][0][g])
    order = 0
    for t in range(fx.T):
        if fx.state(t)["status"][g] != 1:
            break   # the reference game is over (the fixture autoresets; GameUpdater does not)
        res, ups = upd.update(gs, fx.actions[t, g, 0], fx.actions[t, g, 1])
        assert [_as_record(u) for u in ups] == fx.events(t, g), (name, t)
        assert [u.order for u in ups] == list(range(order, order + len(ups)))
        order += len(ups)
        assert int(res) == fx.state(t + 1)["status"][g]
        assert gs == upd.engine.game_states([0])[0], (name, t)
        ents = [(e.iden, e.depth, e.x, e.y, e.health) for e in gs.entities]
        assert ents == fx.entities(t + 1, g), (name, t)
        assert sorted(gs.world.dungeons) == sorted(w[0] for w in fx.world(t + 1, g))


class ReferenceReplayBot:
    """A Bot (optimax_rogue_bots/bot.py interface) that plays back the moves the
    reference's own bots made in a golden fixture, after checking that the view
    BotDriver hands it is the reference's GameState.view_for at that tick:
    tick, its entity, the entities on its depth and that depth's staircase."""

    def __init__(self, fx, g, p):
        self.fx, self.g, self.p, self.t = fx, g, p, 0
        self.checked = 0

    def started(self, gs):
        pass

    def on_move(self, gs, mv):
        self.t += 1

    def finished(self, gs, result):
        pass

    def move(self, gs):
        fx, g, t = self.fx, self.g, self.t
        s = fx.state(t)
        assert gs.tick == int(s["tick"][g]), (fx.name, g, t)
        me = gs.iden_lookup[1 + self.p]
        p = self.p
        assert (me.x, me.y, me.depth, me.health) == (
            int(s["p_x"][p][g]), int(s["p_y"][p][g]), int(s["p_depth"][p][g]),
            int(s["p_health"][p][g])), (fx.name, g, t)
        assert tuple(gs.world.dungeons[me.depth].staircase()) == (
            int(s["st_x"][p][g]), int(s["st_y"][p][g])), (fx.name, g, t)
        want = sorted((e[0], e[2], e[3], e[4]) for e in fx.entities(t, g) if e[1] == me.depth)
        got = sorted((int(e.iden), int(e.x), int(e.y), int(e.health)) for e in gs.entities)
        assert got == want, (fx.name, g, t, got, want)
        self.checked += 1
        return int(fx.actions[t][g][p])


@pytest.mark.parametrize("name", ["c3_npc_64_long", "small_npc_random", "stairs_unused",
                                  "separated_unreachable", "duel_5"])
def test_bot_driver_replays_reference_decisions(name):
    """BotDriver end to end against the reference: every tick each bot
    receives a view equal to the reference's view_for its player (checked by
    the bot), returns the move the reference's RandomBot / StaircaseBot made
    there, and the engine stepped with those moves reproduces the fixture."""
    import torch
    from golden_util import Fixture, compare_state
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.compat import BotDriver
    from optimax_rogue_amd.engine import BatchedEngine
    fx = Fixture(name)
    eng = BatchedEngine(EnvConfig.from_dict(fx.cfg), fx.G, seed=fx.seed,
                        game_offset=fx.game_offset, device=torch.device("cuda", 0))
    bots = [[ReferenceReplayBot(fx, g, p) for g in range(fx.G)] for p in range(2)]
    drv = BotDriver(eng, bots[0], bots[1])
    for _ in range(fx.T):
        drv.step()
    compare_state(eng.snapshot(), fx.state(fx.T), fx.K, f"{name} final")
    assert all(b.checked == fx.T for row in bots for b in row)


@pytest.mark.parametrize("case", ["c3", "stock_npcs", "rpg_all", "dense_npcs", "bank_separated"])
def test_checkpoint_resume(case, tmp_path):
    """save() mid-run, load() into a new engine: both continue bit-identically
    (every state field, including the stock-seed generators, the character
    attributes, items and the dense-NPC occupancy grid)."""
    import torch
    from optimax_rogue_amd import DungeonBank, EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    cfgs = {
        "c3": EnvConfig.c3(),
        "stock_npcs": EnvConfig(width=10, height=9, n_npcs=4, despawn=2, max_ticks=60, rng=1),
        "rpg_all": EnvConfig(width=10, height=9, n_npcs=6, max_ticks=80, flags=4 | 8 | 16 | 32 | 64),
        "dense_npcs": EnvConfig(width=16, height=16, n_npcs=40, npc_health=2, max_ticks=70),
        "bank_separated": EnvConfig(width=12, height=10, n_npcs=3, start_mode=2, p1_depth=2,
                                    p2_depth=0, max_ticks=90,
                                    layouts=DungeonBank.random(12, 10, 5, seed=3).layouts),
    }
    cfg, dev, B = cfgs[case], torch.device("cuda", 0), 2048
    a = BatchedEngine(cfg, B, seed=17, game_offset=5, device=dev)
    a.rollout(100, 2, 1)
    path = str(tmp_path / "ckpt.npz")
    a.save(path)
    b = BatchedEngine.load(path, device=dev)
    for e in (a, b):
        e.rollout(150, 2, 1)
    sa, sb = a.snapshot(), b.snapshot()
    assert sorted(sa) == sorted(sb)
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), (case, k)
    if a.npc_grid is not None:
        assert torch.equal(a.npc_grid, b.npc_grid)


def test_vecenv_step_and_rollout(oracle_lib):
    """VecEnv against the oracle: observations are the state rows, the
    rewards / dones of every step sum to the oracle's episode returns and
    counts; rollout's rewards equal the engine's own return bookkeeping."""
    import torch
    from optimax_rogue_amd import EnvConfig, VecEnv
    cfg = EnvConfig(width=6, height=6, n_npcs=2, max_ticks=25, player_health=3)
    B, dev = 1024, torch.device("cuda", 0)
    env = VecEnv(cfg, B, seed=9, device=dev, opponent=2)     # StaircaseBot opponent
    ora = oracle_lib.Oracle(cfg.to_dict(), B, 9)
    ora.reset(episode=np.ones(B, np.int32))   # env.reset(): every game's next episode (1)
    obs = env.reset()
    rs = np.random.RandomState(2)
    rew_sum = np.zeros(B)
    dones = np.zeros(B, np.int64)
    for t in range(120):
        a1 = rs.randint(1, 6, size=B).astype(np.int8)
        want_a = ora.policy(0, 2, np.stack([a1, np.full(B, 5, np.int8)], 1))
        ora.step(want_a)
        obs, r, d, _ = env.step(torch.from_numpy(a1))
        ex = ora.export()
        want = np.stack([ex["p_x"][0], ex["p_y"][0], ex["p_depth"][0], ex["p_health"][0],
                         ex["p_x"][1], ex["p_y"][1], ex["p_depth"][1], ex["p_health"][1],
                         ex["tick"], ex["status"], ex["st_x"][0], ex["st_y"][0],
                         ex["st_x"][1], ex["st_y"][1]], 1)
        assert np.array_equal(obs.cpu().numpy(), want), t
        rew_sum += r.cpu().numpy()
        dones += d.cpu().numpy()
    ex = ora.export()
    assert np.array_equal(rew_sum, ex["ret_sum"]) and np.array_equal(dones, ex["ep_count"])
    assert dones.sum() > B // 2
    before = env.engine.episode_returns().cpu().numpy().copy()
    out = env.rollout(200, 1, 2)
    after = env.engine.episode_returns().cpu().numpy()
    assert np.array_equal(out["reward"].sum(0).cpu().numpy(), after[0] - before[0])
    assert np.array_equal(out["done"].sum(0).cpu().numpy(), after[1] - before[1])


def test_vecenv_reset_starts_next_episodes(oracle_lib):
    """VecEnv.reset(mask) truncates the masked games into their NEXT episode
    (a fresh dungeon and fresh draws, the oracle's setup of that episode);
    two resets in a row give different starts; the status step() returns is
    a copy the next step does not overwrite."""
    import torch
    from golden_util import compare_state
    from optimax_rogue_amd import EnvConfig, VecEnv
    cfg = EnvConfig.c3()
    B, dev = 2048, torch.device("cuda", 0)
    env = VecEnv(cfg, B, seed=4, device=dev)
    o0 = env.observe().cpu().numpy()
    o1 = env.reset().cpu().numpy()
    o2 = env.reset().cpu().numpy()
    assert (env.engine.episode.cpu().numpy() == 2).all()
    for a, b in ((o0, o1), (o1, o2)):   # positions/staircases of the new episodes differ
        assert (a[:, [0, 1, 4, 5, 10, 11]] != b[:, [0, 1, 4, 5, 10, 11]]).any(1).mean() > 0.99
    ora = oracle_lib.Oracle(cfg.to_dict(), B, 4)
    ora.reset(episode=np.full(B, 2, np.int32))
    compare_state(env.engine.snapshot(), ora.export(), cfg.n_npcs, "two resets")
    # a masked reset advances only the masked games
    for _ in range(7):
        _, _, _, st = env.step(torch.randint(1, 6, (B,), dtype=torch.int8, device=dev))
    st_copy = st.clone()
    env.step(torch.randint(1, 6, (B,), dtype=torch.int8, device=dev))
    assert torch.equal(st, st_copy)
    mask = torch.zeros(B, dtype=torch.bool)
    mask[::3] = True
    ep_before = env.engine.episode.cpu().numpy().copy()
    env.reset(mask)
    ep = env.engine.episode.cpu().numpy()
    m = mask.numpy()
    assert (ep[m] == ep_before[m] + 1).all() and (ep[~m] == ep_before[~m]).all()
    tick = env.engine.tick.cpu().numpy()
    assert (tick[m] == 1).all() and (tick[~m] > 1).all()


@pytest.mark.parametrize("case", ["c3_int64", "selfplay_int32", "stairs_opponent", "dense_bank",
                                  "heal_ext", "sep_double_npc16", "c3_bench", "moving_npcs",
                                  "moving_npcs_dense"])
def test_vecenv_fused_step_equals_policy_step(case):
    """VecEnv.step (one orx_env_step launch, no host sync) against the
    unfused engine calls it replaces -- orx_policy for player 2, orx_step,
    then VecEnv.outcome and observe() on the host side of the comparison --
    for int8..int64 learner actions, self-play, both opponent policies,
    register / dense NPCs, a dungeon bank and the character extensions
    (actions 6 = heal valid), separation damage with double deaths."""
    import torch
    from optimax_rogue_amd import DungeonBank, EnvConfig, VecEnv
    from optimax_rogue_amd.engine import BatchedEngine
    from optimax_rogue_amd.enums import Policy
    dev = torch.device("cuda", 0)
    layouts = None
    if case == "c3_int64":
        cfg, opp, dt, hi = EnvConfig(width=64, height=64, n_npcs=8, max_ticks=40), 1, torch.int64, 5
    elif case == "c3_bench":   # bench.py's vecenv_step extra: C3 at 65,536 games
        cfg, opp, dt, hi = EnvConfig.c3(), 1, torch.int64, 5
    elif case == "sep_double_npc16":
        cfg, opp, dt, hi = EnvConfig(width=9, height=8, n_npcs=14, npc_health=1, max_ticks=0,
                                     start_mode=2, p1_depth=0, p2_depth=1, flags=1 | 2,
                                     sep_period=3, player_health=5), 2, torch.int32, 5
    elif case == "moving_npcs":   # the enemy AI (npc_policy RANDOM), register NPCs
        cfg, opp, dt, hi = EnvConfig(width=9, height=9, n_npcs=12, npc_damage=2, max_ticks=60,
                                     npc_policy=1), 1, torch.int64, 5
    elif case == "moving_npcs_dense":   # CHASE, dense NPCs, StaircaseBot opponent
        cfg, opp, dt, hi = EnvConfig(width=12, height=12, n_npcs=30, npc_health=2, max_ticks=60,
                                     npc_policy=2), 2, torch.int32, 5
    elif case == "selfplay_int32":
        cfg, opp, dt, hi = EnvConfig(width=8, height=7, n_npcs=3, max_ticks=30,
                                     player_health=3), None, torch.int32, 5
    elif case == "stairs_opponent":
        cfg, opp, dt, hi = EnvConfig(width=9, height=9, max_ticks=50, start_mode=2, p1_depth=0,
                                     p2_depth=1), 2, torch.int8, 5
    elif case == "dense_bank":
        bank = DungeonBank.random(12, 10, 4, seed=3, n_stairs=2)
        layouts = bank.layouts
        cfg, opp, dt, hi = EnvConfig(width=12, height=10, n_npcs=24, max_ticks=60,
                                     npc_health=1, layouts=layouts), 1, torch.int16, 5
    else:
        cfg, opp, dt, hi = EnvConfig(width=8, height=8, n_npcs=6, max_ticks=50,
                                     flags=4 | 8 | 16 | 32, player_health=4), 1, torch.int64, 6
    B, T = (65536, 60) if case == "c3_bench" else (1537, 80)
    env = VecEnv(cfg, B, seed=13, device=dev, opponent=opp)
    ref = BatchedEngine(cfg, B, seed=13, device=dev)
    g = torch.Generator(device="cpu").manual_seed(5)
    dones = 0
    for t in range(T):
        shape = (B, 2) if opp is None else (B,)
        a = torch.randint(1, hi + 1, shape, generator=g).to(dt).to(dev)
        obs, r, d, st = env.step(a)
        a8 = a.to(torch.int8)
        if opp is None:
            ref.actions.copy_(a8)
        else:
            ref.actions[:, 0].copy_(a8)
            ref.policy(Policy.NONE, opp)
        before = ref.status.clone()
        want_st = ref.step(ref.actions).clone()
        want_r, want_d = VecEnv.outcome(before, want_st)
        assert torch.equal(env.engine.actions, ref.actions), (case, t)
        assert torch.equal(st, want_st), (case, t)
        assert torch.equal(d, want_d) and torch.equal(r, want_r), (case, t)
        e = ref
        want_obs = torch.stack([e.p_x[0], e.p_y[0], e.p_depth[0], e.p_health[0], e.p_x[1],
                                e.p_y[1], e.p_depth[1], e.p_health[1], e.tick, e.status,
                                e.st_x[0], e.st_y[0], e.st_x[1], e.st_y[1]], dim=1)
        assert torch.equal(obs, want_obs), (case, t)
        dones += int(d.sum())
    assert case == "c3_bench" or dones > B // 4, case   # (C3's 1,000-tick episodes: none end)
    a, b = env.engine.snapshot(), ref.snapshot()
    for k in a:
        assert np.array_equal(a[k], b[k]), (case, k)


@pytest.mark.parametrize("cfgname,B", [("c3", 65536), ("npc_small", 1537), ("dense", 999),
                                       ("moving", 777)])
def test_env_step_games_per_wave_invariance(cfgname, B, monkeypatch):
    """orx_env_step at 64 and at 32 games per wave (ORX_ENV_LANES: two
    half-full waves per SIMD) gives identical outputs and state, batch sizes
    that leave a partial workgroup included (its LDS row run)."""
    import torch
    from optimax_rogue_amd import EnvConfig, VecEnv
    cfg = {"c3": EnvConfig.c3(), "npc_small": EnvConfig(width=9, height=8, n_npcs=5, max_ticks=30),
           "dense": EnvConfig(width=12, height=12, n_npcs=20, max_ticks=40),
           "moving": EnvConfig(width=9, height=9, n_npcs=6, max_ticks=40, npc_policy=1)}[cfgname]
    dev = torch.device("cuda", 0)
    res = []
    for lanes in ("64", "32"):
        monkeypatch.setenv("ORX_ENV_LANES", lanes)
        env = VecEnv(cfg, B, seed=21, device=dev, opponent=1)
        g = torch.Generator(device="cpu").manual_seed(2)
        outs = []
        for t in range(30):
            a = torch.randint(1, 6, (B,), generator=g, dtype=torch.int64).to(dev)
            outs.append([x.cpu() for x in env.step(a)])
        res.append((outs, env.engine.snapshot()))
    (o64, s64), (o32, s32) = res
    for t, (a, b) in enumerate(zip(o64, o32)):
        for x, y in zip(a, b):
            assert torch.equal(x, y), (cfgname, t)
    for k in s64:
        assert np.array_equal(s64[k], s32[k]), (cfgname, k)


@pytest.mark.parametrize("cfgname,B", [("random16", 1537), ("chase8", 999), ("dense", 333),
                                       ("stock", 257)])
def test_moving_rollout_games_per_wave_invariance(cfgname, B, monkeypatch):
    """mov_rollout_kernel at 64, 16 and 1 games per wave (ORX_MOV_LANES)
    writes identical rows and actions and leaves identical state, with
    partial waves and workgroups, autoresets inside the launch, dense NPCs
    and stock-seed mode."""
    import torch
    from optimax_rogue_amd import EnvConfig, OBS_FIELDS, Policy
    from optimax_rogue_amd.engine import BatchedEngine
    cfg = {"random16": EnvConfig(width=12, height=12, n_npcs=16, max_ticks=30, npc_policy=1),
           "chase8": EnvConfig(width=10, height=9, n_npcs=8, max_ticks=25, npc_policy=2),
           "dense": EnvConfig(width=12, height=12, n_npcs=20, max_ticks=30, npc_policy=1),
           "stock": EnvConfig(width=10, height=10, n_npcs=5, max_ticks=30, npc_policy=1,
                              rng=1)}[cfgname]
    dev = torch.device("cuda", 0)
    T = 70
    res = []
    for lanes in ("64", "16", "1"):
        monkeypatch.setenv("ORX_MOV_LANES", lanes)
        eng = BatchedEngine(cfg, B, seed=8, device=dev)
        obs = torch.empty((T, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
        act = torch.empty((T, B, 2), dtype=torch.int8, device=dev)
        eng.rollout(T, Policy.Random, Policy.Random, obs=obs, act=act)
        res.append((obs.cpu(), act.cpu(), eng.snapshot()))
    base = res[0]
    assert int(base[2]["episode"].sum()) > 0   # autoresets happened
    for r in res[1:]:
        assert torch.equal(r[0], base[0]) and torch.equal(r[1], base[1]), cfgname
        for k in base[2]:
            assert np.array_equal(r[2][k], base[2][k]), (cfgname, k)


def test_vecenv_bad_actions_truncate_on_device():
    """Values outside the Move codes (0, -1, 6 without EXT_HEAL, 257 as
    int64 -- which an int8 cast would wrap to the legal 1 -- and 128..255 as
    uint8) stop exactly
    those games with STATUS_BAD_ACTION: done, reward 0, no host sync; the
    next step starts their next episode.  check_actions=True raises instead."""
    import torch
    from optimax_rogue_amd import EnvConfig, VecEnv
    from optimax_rogue_amd.enums import STATUS_BAD_ACTION
    dev = torch.device("cuda", 0)
    B = 512
    env = VecEnv(EnvConfig(width=10, height=10, max_ticks=100), B, seed=2, device=dev)
    a = torch.full((B,), 5, dtype=torch.int64, device=dev)
    bad = {3: 0, 10: -1, 77: 6, 100: 257, 511: 1 << 40}
    for k, v in bad.items():
        a[k] = v
    ep0 = env.engine.episode.clone()
    obs, r, d, st = env.step(a)
    idx = torch.tensor(sorted(bad), device=dev)
    assert (st[idx] == STATUS_BAD_ACTION).all() and d[idx].all() and (r[idx] == 0).all()
    keep = torch.ones(B, dtype=torch.bool, device=dev)
    keep[idx] = False
    assert (st[keep] == 1).all() and not d[keep].any()
    assert (obs[:, 9] == st).all()
    obs, r, d, st = env.step(torch.full((B,), 5, dtype=torch.int8, device=dev))
    assert (st == 1).all() and not d.any()
    ep = env.engine.episode
    assert (ep[idx] == ep0[idx] + 1).all() and (ep[keep] == ep0[keep]).all()
    assert (obs[idx, 8] == 1).all()   # their next episode's first tick
    # uint8 learner actions (read as int8): 0 and 128..255 are refused
    u = torch.full((B,), 2, dtype=torch.uint8, device=dev)
    ubad = {5: 0, 6: 128, 9: 255}
    for k, v in ubad.items():
        u[k] = v
    obs, r, d, st = env.step(u)
    uidx = torch.tensor(sorted(ubad), device=dev)
    ukeep = torch.ones(B, dtype=torch.bool, device=dev)
    ukeep[uidx] = False
    assert (st[uidx] == STATUS_BAD_ACTION).all() and d[uidx].all()
    assert (st[ukeep] == 1).all() and not d[ukeep].any()
    strict = VecEnv(EnvConfig(width=10, height=10), 8, seed=2, device=dev, check_actions=True)
    with pytest.raises(ValueError, match="Move values"):
        strict.step(torch.tensor([1, 2, 3, 4, 5, 0, 1, 1], device=dev))


def test_vecenv_deferred_bad_action_check():
    """The default check_actions="deferred": refused actions are counted on
    the device by orx_env_step_ex (no host sync) and a later step warns once
    the asynchronous read-back shows them (every tick is still played);
    "deferred-raise" raises ValueError instead.  Correct actions never report,
    a report is not repeated for the same refusals, bad_actions() reads the
    count."""
    import warnings
    import torch
    from optimax_rogue_amd import EnvConfig, VecEnv
    dev = torch.device("cuda", 0)
    B = 256
    for mode in ("deferred", "deferred-raise"):
        env = VecEnv(EnvConfig(width=10, height=10, max_ticks=50), B, seed=5, device=dev,
                     check_every=4, **({} if mode == "deferred" else {"check_actions": mode}))
        good = torch.full((B,), 2, dtype=torch.int64, device=dev)
        for _ in range(40):
            env.step(good)
        assert env.bad_actions() == 0
        bad = good.clone()
        bad[[1, 7, 200]] = 0                       # a 0-based argmax in three games
        env.step(bad)
        raised = 0
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            for _ in range(60):
                try:
                    env.step(good)
                except ValueError as e:
                    assert "3 game(s)" in str(e) and "0-based" in str(e)
                    raised += 1
                torch.cuda.synchronize()
        msgs = [str(x.message) for x in w if issubclass(x.category, RuntimeWarning)]
        if mode == "deferred":
            assert raised == 0 and len(msgs) == 1 and "3 game(s)" in msgs[0]
            assert env.warnings_seen == 1
        else:
            assert raised == 1 and not msgs
        assert env.bad_actions() == 3


def test_vecenv_check_actions_normalized():
    """check_actions accepts bools (1 / numpy True mean the host check), the
    two deferred modes, and nothing else."""
    import numpy as np
    import torch
    from optimax_rogue_amd import EnvConfig, VecEnv
    dev = torch.device("cuda", 0)
    cfg = EnvConfig(width=10, height=10)
    for v in (1, np.True_, True):
        env = VecEnv(cfg, 8, seed=2, device=dev, check_actions=v)
        assert env.check_actions is True
        with pytest.raises(ValueError, match="Move values"):
            env.step(torch.tensor([1, 2, 3, 4, 5, 0, 1, 1], device=dev))
    assert VecEnv(cfg, 8, device=dev, check_actions=np.False_).check_actions is False
    for v in ("raise", 2, None):
        with pytest.raises(ValueError, match="check_actions"):
            VecEnv(cfg, 8, device=dev, check_actions=v)


def test_vecenv_out_buffers_ring():
    """out_buffers=k: the same results as fresh tensors, from a ring of k
    preallocated sets (step t's tensors are step t+k's)."""
    import torch
    from optimax_rogue_amd import EnvConfig, VecEnv
    dev = torch.device("cuda", 0)
    B = 1000
    cfg = EnvConfig(width=8, height=8, n_npcs=3, max_ticks=30, player_health=3)
    fresh = VecEnv(cfg, B, seed=8, device=dev)
    ring = VecEnv(cfg, B, seed=8, device=dev, out_buffers=3)
    g = torch.Generator(device="cpu").manual_seed(1)
    ptrs = []
    for t in range(20):
        a = torch.randint(1, 6, (B,), generator=g).to(dev)
        want = [x.clone() for x in fresh.step(a)]
        got = ring.step(a)
        for w, x in zip(want, got):
            assert torch.equal(w, x), t
        ptrs.append(got[0].data_ptr())
    assert len(set(ptrs)) == 3 and ptrs[0] == ptrs[3] == ptrs[6]
