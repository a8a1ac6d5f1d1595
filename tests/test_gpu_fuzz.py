"""GPU parity over seeded random configurations: the engine against the C
oracle on configurations drawn from the whole orx_cfg_t space at once
(grid shape, despawn rule, start mode and depths, max_ticks, NPC count in the
register and dense forms, combat attributes, dungeon bank, stock seeding,
every build-extension flag, moving NPCs, games per rollout wave), so feature
combinations
no hand-written case names are exercised too.

Each configuration runs twice against the oracle from the same reset:
  * per tick: uniformly random actions (heals included when EXT_HEAL is on)
    through ``orx_step`` -- the reference's ``Updater.update`` per tick
    (updater.py:76-162);
  * fused: ``orx_rollout`` with a random pair of device bots (RandomBot /
    StaircaseBot, randombot.py:20-21, staircasebot.py:9-21) against the
    oracle's policy + step, with the trajectory rows and actions compared.
Bit-exact (all state is integer).  Reference-pinned where the configuration
stays inside the reference's semantics (flags 0); engine-vs-oracle only
("parity unpinned") where a build extension is on.  The generator is seeded,
so a failure names a reproducible case id.
"""
import os

import numpy as np
import pytest

from golden_util import compare_state

# ORX_FUZZ_CASES / ORX_FUZZ_BASE widen or move the sweep for ad-hoc runs
N_CASES = int(os.environ.get("ORX_FUZZ_CASES", "96"))
BASE = int(os.environ.get("ORX_FUZZ_BASE", "1000"))
MANA, HEAL, LEVEL, ITEMS, README = 4, 8, 16, 32, 64


def _layouts(rs, W, H):
    """A small explicit-grid bank: walls ~0-25%, some open edges, 1-3 staircases."""
    L = int(rs.randint(1, 7))
    out = []
    for li in range(L):
        t = np.ones((W, H), np.uint8)
        t[[0, -1], :] = 2
        t[:, [0, -1]] = 2
        if rs.rand() < 0.3:
            t[0, 1:H - 1] = 1
        inner = rs.rand(W, H) < rs.uniform(0, 0.25)
        inner[[0, -1], :] = False
        inner[:, [0, -1]] = False
        t[inner] = 2
        g = np.argwhere(t == 1)
        for j in rs.choice(len(g), int(rs.randint(1, 4)), replace=False):
            t[tuple(g[j])] = 3
        out.append(t)
    return np.stack(out)


def _draw(case: int, base: int = None):
    """Configuration, layouts, batch, ticks, seed, offset, bots, lanes of case."""
    rs = np.random.RandomState((BASE if base is None else base) + case)
    W, H = int(rs.randint(4, 40)), int(rs.randint(4, 40))
    if rs.rand() < 0.15:
        W, H = int(rs.choice([64, 96, 128])), int(rs.choice([64, 128]))
    cfg = dict(width=W, height=H, despawn=int(rs.choice([1, 2])),
               max_ticks=int(rs.choice([0, 15, 40, 120, 1000])),
               player_health=int(rs.randint(1, 14)), player_damage=int(rs.randint(1, 5)),
               player_armor=int(rs.randint(0, 3)))
    if rs.rand() < 0.35:
        d1 = int(rs.randint(0, 4))
        cfg.update(start_mode=2, p1_depth=d1, p2_depth=int((d1 + rs.randint(1, 4)) % 5))
        if cfg["p2_depth"] == d1:
            cfg["p2_depth"] = d1 + 1
    layouts = _layouts(rs, W, H) if rs.rand() < 0.3 and min(W, H) >= 6 else None
    if layouts is not None and (layouts == 1).sum(axis=(1, 2)).min() < 4:
        layouts = None
    # NPCs: none, register slots (<= 16) or the dense occupancy-grid form,
    # leaving Ground for both players (engine.py refuses a bank without it)
    room = ((W - 2) * (H - 2) - 3 if layouts is None
            else int((layouts == 1).sum(axis=(1, 2)).min()) - 3)
    kind = rs.rand()
    if kind < 0.25:
        K = 0
    elif kind < 0.75:
        K = int(rs.randint(1, 17))
    else:
        K = int(rs.randint(17, 64 if rs.rand() < 0.8 else 256))
    K = min(K, max(0, room))
    cfg.update(n_npcs=K, npc_health=int(rs.choice([1, 2, 3, 4, 127])), npc_damage=int(rs.randint(0, 3)),
               npc_armor=int(rs.randint(0, 2)))
    flags = 0
    if rs.rand() < 0.5:
        for f, p in ((1, 0.3), (2, 0.3), (MANA, 0.3), (LEVEL, 0.3), (README, 0.25)):
            if rs.rand() < p:
                flags |= f
        if flags & MANA and rs.rand() < 0.5:
            flags |= HEAL
        if K <= 16 and rs.rand() < 0.3:
            flags |= ITEMS
    cfg.update(flags=flags, sep_period=int(rs.randint(1, 9)), mana_max=int(rs.randint(3, 13)),
               mana_regen=int(rs.randint(0, 3)), mana_per_point=int(rs.randint(1, 3)),
               xp_per_kill=int(rs.randint(0, 3)), xp_per_level=int(rs.randint(1, 4)),
               item_drop_pct=int(rs.randint(0, 101)), item_bonus=int(rs.randint(0, 3)),
               item_slots=int(rs.randint(0, 4)), combat_cooldown=int(rs.randint(0, 4)))
    if W <= 256 and H <= 256 and rs.rand() < 0.2:
        cfg["rng"] = 1
    # moving NPCs (round 6): the enemy AI on about a third of the configurations
    # it supports (NPCs, flags within separation damage and double death),
    # drawn from a stream of its own so the other draws stay as they were
    mv = np.random.RandomState(((BASE if base is None else base) + case) ^ 0x5EED)
    if K > 0 and not (flags & ~3) and mv.rand() < 0.35:
        cfg["npc_policy"] = int(mv.choice([1, 2]))
    B = int(rs.choice([1, 63, 257, 1000, 1531]))
    T = int(rs.randint(40, 161))
    pol = (int(rs.choice([1, 1, 2, 2, 3])), int(rs.choice([1, 1, 2, 2, 3])))
    lanes = int(rs.choice([0, 0, 64, 32, 16, 8]))
    return cfg, layouts, B, T, int(rs.randint(0, 2 ** 31)), int(rs.randint(0, 5000)), pol, lanes


def test_draws_are_valid_and_varied(oracle_lib):
    """Every drawn configuration satisfies orx_validate_cfg's rules and runs on
    the oracle; together the draws cover every feature the sweep is for."""
    seen = set()
    for c in range(N_CASES):
        cfg, layouts, B, T, seed, off, pol, lanes = _draw(c)
        assert cfg["width"] >= 4 and cfg["height"] >= 4
        assert not cfg["flags"] & ITEMS or cfg["n_npcs"] <= 16
        assert not cfg["flags"] & HEAL or cfg["flags"] & MANA
        if layouts is not None:
            assert (layouts == 1).sum(axis=(1, 2)).min() >= cfg["n_npcs"] + 2
        else:
            assert (cfg["width"] - 2) * (cfg["height"] - 2) - 1 >= cfg["n_npcs"] + 2
        o = oracle_lib.Oracle(cfg, min(B, 64), seed, off, layouts=layouts)
        o.reset(episode=np.zeros(min(B, 64), np.int32))
        for _ in range(5):
            o.step(o.policy(*pol))
        K = cfg["n_npcs"]
        seen |= {"bank"} if layouts is not None else set()
        seen |= {"dense"} if K > 16 else ({"npcs"} if K else set())
        seen |= {"separated"} if cfg.get("start_mode") == 2 else set()
        seen |= {"stock"} if cfg.get("rng") else set()
        seen |= {f"flag{f}" for f in (1, 2, MANA, HEAL, LEVEL, ITEMS, README) if cfg["flags"] & f}
        seen |= {"plain"} if not cfg["flags"] else set()
        seen |= {f"moving{cfg['npc_policy']}"} if cfg.get("npc_policy") else set()
    want = {"bank", "dense", "npcs", "separated", "stock", "plain", "flag1", "flag2",
            "flag4", "flag16", "flag32", "flag64", "moving1", "moving2"}
    assert want <= seen, want - seen


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(N_CASES))
def test_random_config_vs_oracle(case, oracle_lib, monkeypatch):
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    from optimax_rogue_amd.enums import OBS_FIELDS
    cfg, layouts, B, T, seed, off, pol, lanes = _draw(case)
    where = f"case {case} {cfg} B={B} T={T} pol={pol} lanes={lanes} bank={layouts is not None}"
    if lanes:
        monkeypatch.setenv("ORX_ROLLOUT_LANES", str(lanes))
    dev = torch.device("cuda", 0)

    def pair():
        o = oracle_lib.Oracle(cfg, B, seed, off, layouts=layouts)
        o.reset(episode=np.zeros(B, np.int32))
        e = BatchedEngine(EnvConfig.from_dict(cfg, layouts=layouts), B, seed=seed,
                          game_offset=off, device=dev)
        compare_state(e.snapshot(), o.export(), o.K, f"{where} reset")
        return o, e

    # per tick, random actions through orx_step_events: state, and the update
    # events of a few games every tick
    ora, eng = pair()
    ora = oracle_lib.Oracle(cfg, B, seed, off, layouts=layouts, record_events=True)
    ora.reset(episode=np.zeros(B, np.int32))
    rs = np.random.RandomState(seed % 100003)
    hi = 7 if cfg["flags"] & HEAL else 6
    for t in range(T):
        a = rs.randint(1, hi, size=(B, 2)).astype(np.int8)
        ora.step(a)
        _, ev, nev = eng.step(torch.from_numpy(a).to(dev).contiguous(), events=True)
        ev, nev = ev.cpu().numpy(), nev.cpu().numpy()
        for g in rs.randint(0, B, size=3):
            got = [tuple(int(v) for v in r) for r in ev[g, : nev[g]]]
            assert got == ora.events(int(g)), f"{where} events t={t + 1} game {g}"
        if t % 40 == 39 or t == T - 1:
            compare_state(eng.snapshot(), ora.export(), ora.K, f"{where} step t={t + 1}")

    # fused rollout with device bots, in three launches
    ora, eng = pair()
    n = max(1, T // 3)
    obs = torch.zeros((n, len(OBS_FIELDS), B), dtype=torch.int32, device=dev)
    act = torch.zeros((n, B, 2), dtype=torch.int8, device=dev)
    for c in range(3):
        want_act, want_obs = [], []
        for _ in range(n):
            a = ora.policy(*pol)
            ora.step(a)
            want_act.append(a)
            s = ora.export()
            want_obs.append(np.stack([s["p_x"][0], s["p_y"][0], s["p_depth"][0], s["p_health"][0],
                                      s["p_x"][1], s["p_y"][1], s["p_depth"][1], s["p_health"][1],
                                      s["tick"], s["status"], s["st_x"][0], s["st_y"][0],
                                      s["st_x"][1], s["st_y"][1]]))
        eng.rollout(n, *pol, obs=obs, act=act)
        compare_state(eng.snapshot(), ora.export(), ora.K, f"{where} rollout launch {c}")
        assert np.array_equal(act.cpu().numpy(), np.stack(want_act)), f"{where} actions {c}"
        assert np.array_equal(obs.cpu().numpy(), np.stack(want_obs)), f"{where} obs {c}"
    torch.cuda.synchronize()


N_SEQ = int(os.environ.get("ORX_FUZZ_SEQ", "32"))


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(N_SEQ))
def test_random_call_sequence_vs_oracle(case, oracle_lib, monkeypatch, tmp_path):
    """State hand-over between the entry points: a seeded random sequence of
    orx_step (given actions), orx_policy + orx_step, orx_rollout of 1-40 ticks,
    orx_step_n replaying a 1-40 tick move log (about 1% of its moves outside
    the Move codes; keyed streams only), masked orx_reset into a chosen
    episode and checkpoint/resume (save -> load into a new engine) on one
    random configuration, against the oracle doing the same, compared after
    every call."""
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    cfg, layouts, B, T, seed, off, pol, lanes = _draw(7919 + case)
    where = f"seq {case} {cfg} B={B} lanes={lanes} bank={layouts is not None}"
    if lanes:
        monkeypatch.setenv("ORX_ROLLOUT_LANES", str(lanes))
    dev = torch.device("cuda", 0)
    ora = oracle_lib.Oracle(cfg, B, seed, off, layouts=layouts)
    ora.reset(episode=np.zeros(B, np.int32))
    eng = BatchedEngine(EnvConfig.from_dict(cfg, layouts=layouts), B, seed=seed,
                        game_offset=off, device=dev)
    rs = np.random.RandomState(case)
    hi = 7 if cfg["flags"] & HEAL else 6
    log = []
    for j in range(24):
        op = rs.choice(["step", "policy", "rollout", "replay", "reset", "resume"],
                       p=[.2, .15, .3, .15, .12, .08])
        p = (int(rs.choice([1, 2, 3])), int(rs.choice([1, 2, 3])))
        if op == "replay" and cfg.get("rng"):
            op = "step"   # (orx_step_n refuses stock-seed mode)
        if op == "step":
            a = rs.randint(1, hi, size=(B, 2)).astype(np.int8)
            ora.step(a)
            eng.step(torch.from_numpy(a).to(dev).contiguous())
        elif op == "policy":
            a = ora.policy(*p)
            ora.step(a)
            got = eng.policy(*p)
            assert np.array_equal(got.cpu().numpy(), a), f"{where} {log} policy"
            eng.step(got)
        elif op == "replay":
            n = int(rs.randint(1, 41))
            acts = rs.randint(1, hi, size=(n, B, 2)).astype(np.int8)
            bad = rs.rand(n, B, 2) < 0.01
            acts[bad] = rs.choice([0, -1, hi, 99], size=int(bad.sum())).astype(np.int8)
            for t in range(n):
                ora.step(acts[t])
            eng.step_n(torch.from_numpy(acts).to(dev).contiguous())
            op = f"replay{n}"
        elif op == "rollout":
            n = int(rs.randint(1, 41))
            for _ in range(n):
                ora.step(ora.policy(*p))
            eng.rollout(n, *p)
            op = f"rollout{n}"
        elif op == "reset":
            mask = rs.rand(B) < rs.choice([0.1, 0.5, 1.0])
            ep = rs.randint(0, 1000, size=B).astype(np.int32)
            cur = eng.snapshot()["episode"]
            ep = np.where(mask, ep, cur).astype(np.int32)
            ora.reset(mask=mask, episode=ep)
            eng.reset(torch.from_numpy(mask), episode=torch.from_numpy(ep))
        else:
            path = tmp_path / f"ck{j}.npz"
            eng.save(path)
            eng = BatchedEngine.load(path, device=dev)
        log.append(op)
        compare_state(eng.snapshot(), ora.export(), ora.K, f"{where} after {log}")
    torch.cuda.synchronize()
