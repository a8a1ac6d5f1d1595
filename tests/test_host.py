"""CPU: host-side helpers that need no GPU (the engine itself is tested
with -m gpu)."""
import numpy as np
import pytest


def test_vecenv_outcome():
    """reward / done of a status transition: only games in progress before
    the step that end in it count; player 1's view."""
    torch = pytest.importorskip("torch")
    from optimax_rogue_amd.vecenv import VecEnv
    before = torch.tensor([1, 1, 1, 1, 2, 3, 4, 16, 1, 1, 16], dtype=torch.int32)
    after = torch.tensor([1, 2, 3, 4, 1, 3, 4, 16, 16, 17, 1], dtype=torch.int32)
    reward, done = VecEnv.outcome(before, after)
    # an engine stop code (>= 16) ends the episode as a truncation (reward 0):
    # the autoreset restarts the game on the next step
    assert done.tolist() == [False, True, True, True, False, False, False, False, True, True,
                             False]
    assert reward.tolist() == [0.0, 1.0, -1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0]


@pytest.mark.parametrize("bad", [[0, 1, 2], [1, 6, 2], [1, 2, 257], [-1, 2, 3]])
def test_vecenv_step_rejects_non_moves(bad):
    """check_actions=True: a learner's 0-based argmax (or any value outside
    the Move codes) is refused on the host before it reaches the engine."""
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.vecenv import VecEnv
    env = VecEnv.__new__(VecEnv)
    env.engine = _bare_engine(EnvConfig(), 3)
    env.B, env.device, env.opponent, env.check_actions = 3, torch.device("cpu"), 1, True
    env.check_every, env.out_buffers = 64, 0
    env._init_step_consts()
    with pytest.raises(ValueError, match="Move values"):
        env.step(torch.tensor(bad, dtype=torch.int32))
    with pytest.raises(ValueError, match="Move values"):
        env.step(torch.tensor([bad, bad, bad], dtype=torch.int64).t().contiguous()[:, :2])
    # with EXT_HEAL, 6 (a heal) is a valid action
    env.engine.cfg = EnvConfig(flags=4 | 8)
    assert env._max_move() == 6


def test_npc_alive_bits():
    from optimax_rogue_amd.enums import npc_alive_bits
    a = np.array([0b101, 0xFFFFFFFF], np.uint32)
    bits = npc_alive_bits(a, 3)
    assert bits.shape == (3, 2)
    assert bits[:, 0].tolist() == [True, False, True] and bits[:, 1].all()
    rows = np.zeros((2, 3), np.uint32)       # K = 40: two rows of 32
    rows[1, 2] = 1 << 7                      # NPC 39 of game 2
    rows[0, 0] = 1 << 31                     # NPC 31 of game 0
    b = npc_alive_bits(rows, 40)
    assert b.shape == (40, 3)
    assert sorted(zip(*np.nonzero(b))) == [(31, 0), (39, 2)]


def test_env_config_round_trip():
    """EnvConfig <-> dict <-> the orx_cfg_t mirror keeps every field."""
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.config import CFG_FIELDS
    c = EnvConfig(width=40, height=12, n_npcs=30, flags=4 | 16 | 64, mana_max=12,
                  combat_cooldown=5, item_slots=2, rng=1)
    d = c.to_dict()
    assert set(d) == set(CFG_FIELDS)
    c2 = EnvConfig.from_dict(d)
    assert c2.to_dict() == d
    cc = c.to_c()
    assert [getattr(cc, f) for f in CFG_FIELDS] == [d[f] for f in CFG_FIELDS]


def test_dungeon_bank_random_is_valid():
    from optimax_rogue_amd import DungeonBank
    bank = DungeonBank.random(12, 10, 5, seed=3, n_stairs=2)
    assert bank.layouts.shape == (5, 12, 10)
    for lay in bank.layouts:
        assert (lay == 3).sum() == 2                  # two staircases
        assert (lay[[0, -1], :] == 2).all() and (lay[:, [0, -1]] == 2).all()
    assert bank.min_ground >= 2


def _bare_engine(cfg, B):
    """A BatchedEngine shell with no device state: enough for its host checks."""
    import torch
    from optimax_rogue_amd.engine import BatchedEngine
    e = BatchedEngine.__new__(BatchedEngine)
    e.cfg, e.B, e.K, e.bank, e.device = cfg, B, int(cfg.n_npcs), None, torch.device("cpu")
    return e


def test_engine_refuses_action_buffers_it_would_overrun():
    import torch
    from optimax_rogue_amd import EnvConfig
    e = _bare_engine(EnvConfig.c2(), 8)
    e._check_actions(torch.zeros((8, 2), dtype=torch.int8), "actions")
    for bad in (torch.zeros((4, 2), dtype=torch.int8), torch.zeros((8, 2), dtype=torch.int32),
                torch.zeros((2, 8), dtype=torch.int8).t(), torch.zeros(16, dtype=torch.int8)):
        with pytest.raises(ValueError):
            e._check_actions(bad, "actions")


def test_engine_refuses_snapshots_off_the_grid():
    from optimax_rogue_amd import EnvConfig
    cfg = EnvConfig(width=8, height=6, n_npcs=2)
    e = _bare_engine(cfg, 3)
    ok = {"p_x": np.full((2, 3), 7), "p_y": np.full((2, 3), 5), "p_depth": np.zeros((2, 3)),
          "npc_pos": np.array([[7 | 5 << 8] * 3, [0] * 3]), "npc_alive": np.full(3, 3)}
    e._check_snapshot(ok)
    for key, val in (("p_x", np.full((2, 3), 8)), ("p_y", np.full((2, 3), -1)),
                     ("npc_pos", np.array([[8] * 3, [0] * 3]))):
        with pytest.raises(ValueError):
            e._check_snapshot(dict(ok, **{key: val}))
    # a dead NPC's slot is not read: any position passes
    e._check_snapshot(dict(ok, npc_pos=np.array([[200] * 3, [0] * 3]), npc_alive=np.full(3, 2)))


@pytest.mark.parametrize("bad", [[0, 1, 2], [1, 2, 257], [-1, 2, 3]])
@pytest.mark.parametrize("ring", [0, 2])
def test_vecenv_step_passes_bad_actions_to_the_engine(bad, ring):
    """check_actions=False: no host check and no sync -- the learner's tensor
    goes to the learner-tick launch (orx_env_step_args) as it is (its own
    pointer at full width: 257 is
    not cast to int8, where it would wrap to a legal 1); the engine stops
    those games with STATUS_BAD_ACTION and step() reports them done (GPU
    tests: test_vecenv_bad_actions_truncate_on_device).  Status is its own
    tensor (not a view of the observation); with out_buffers=k the outputs
    come from a ring of k sets."""
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.vecenv import VecEnv
    calls = []

    class Eng:
        cfg, mt_py = EnvConfig(), None

        def env_step_slot(self, p2, obs, rew, done, status, bad=None):
            # (BatchedEngine.env_step_slot: a launch over one argument block)
            ptrs = (obs.data_ptr(), rew.data_ptr(), done.data_ptr(), status.data_ptr())

            def launch(a_ptr, nb, cols, outs=None):
                o = ptrs if outs is None else outs
                calls.append((a_ptr, nb, cols, p2, *o, None if bad is None else bad.data_ptr()))
            return launch

    env = VecEnv.__new__(VecEnv)
    env.engine, env.check_actions = Eng(), False
    env.B, env.device, env.opponent = 3, torch.device("cpu"), 2
    env.check_every, env.out_buffers = 64, ring
    env._init_step_consts()
    a = torch.tensor(bad, dtype=torch.int64)
    outs = [env.step(a) for _ in range(3)]
    a_ptr, nb, cols, p2, optr, rptr, dptr, sptr, bptr = calls[0]
    assert a_ptr == a.data_ptr() and nb == 8 and cols == 1 and p2 == 2 and bptr is None
    obs, reward, done, status = outs[0]
    assert (optr, rptr, dptr, sptr) == (obs.data_ptr(), reward.data_ptr(), done.data_ptr(),
                                        status.data_ptr())
    assert obs.shape == (3, 14) and obs.dtype == torch.int32 and reward.dtype == torch.float32
    assert done.dtype == torch.bool and status.dtype == torch.int32 and status.shape == (3,)
    assert status.data_ptr() != obs[:, 9].data_ptr()
    same = outs[2][0].data_ptr() == outs[0][0].data_ptr()
    assert same == (ring == 2)   # the ring of two comes round on the third step
    with pytest.raises(ValueError, match="integer"):
        env.step(torch.tensor([1.0, 2.0, 3.0]))


def _encode_compact(rows):
    """The compact encoding of int32 rows [T, 14, B], restated in numpy
    (include/orx.h ORX_OBS_COMPACT)."""
    r = rows.astype(np.int64)
    cell = lambda x, y: (x & 0xFF) | ((y & 0xFF) << 8)
    w = np.stack([cell(r[:, 0], r[:, 1]) | (cell(r[:, 4], r[:, 5]) << 16),
                  cell(r[:, 10], r[:, 11]) | (cell(r[:, 12], r[:, 13]) << 16),
                  (r[:, 3] & 0xFFFF) | ((r[:, 7] & 0xFFFF) << 16), r[:, 2] & 0xFFFFFFFF,
                  r[:, 6] & 0xFFFFFFFF, r[:, 8] | (r[:, 9] << 27)], axis=1)
    return w.astype(np.uint32).view(np.int32)


def test_decode_compact_round_trip():
    """decode_compact inverts the compact encoding over the fields' full
    ranges: cells and staircases 0..255, healths -32768..32767, depths to
    2^31-1, ticks to 2^27-1, every status code."""
    import torch
    from optimax_rogue_amd.engine import decode_compact
    rs = np.random.RandomState(0)
    T, B = 3, 4000
    rows = np.zeros((T, 14, B), np.int64)
    for f in (0, 1, 4, 5, 10, 11, 12, 13):
        rows[:, f] = rs.randint(0, 256, (T, B))
    for f in (3, 7):
        rows[:, f] = rs.randint(-32768, 32768, (T, B))
    for f in (2, 6):
        rows[:, f] = rs.randint(0, 2**31 - 1, (T, B))
    rows[:, 8] = rs.randint(0, 2**27, (T, B))
    rows[:, 9] = rs.choice([1, 2, 3, 4, 16, 17], (T, B))
    got = decode_compact(torch.from_numpy(_encode_compact(rows))).numpy()
    assert got.dtype == np.int32 and np.array_equal(got, rows.astype(np.int32))


def test_compact_rows_refuse_what_does_not_fit(engine_lib):
    """orx_rollout_ex(ORX_OBS_COMPACT) refuses configurations whose values
    the compact fields cannot hold, before any device work."""
    import ctypes
    from optimax_rogue_amd import EnvConfig, _lib
    from optimax_rogue_amd.enums import OBS_COMPACT
    lib = engine_lib
    st = _lib.OrxState()

    def rc(cfg, fmt=OBS_COMPACT):
        return lib.orx_rollout_ex(ctypes.byref(cfg.to_c()), ctypes.byref(st), 1, 1, 4, None,
                                  None, fmt, 8, 1, 0, 1, None)
    for bad in (EnvConfig(width=300, height=20), EnvConfig(max_ticks=0),
                EnvConfig(max_ticks=1 << 27), EnvConfig(player_health=9000),
                EnvConfig(flags=1, sep_period=1, max_ticks=9000),
                EnvConfig(n_npcs=2, npc_damage=20000)):
        assert rc(bad) == -22, bad
        assert "compact" in lib.orx_last_error().decode()
    assert rc(EnvConfig(), fmt=7) == -22
    # a fitting configuration passes the format checks (then fails on the NULL state)
    assert rc(EnvConfig.c3()) == -22 and "compact" not in lib.orx_last_error().decode()
