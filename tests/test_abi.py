"""CPU: the C-ABI library loads, exports every symbol include/orx.h declares,
its POD layouts match the ctypes mirrors, and it is callable from plain C.
No compute runs here (no GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "orx.h")


def header_text():
    return open(HEADER).read()


def declared_functions():
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(orx_\w+)\s*\(", header_text(), re.M)))


def struct_fields(name):
    body = re.search(r"typedef struct %s \{(.*?)\} %s_t;" % (name, name), header_text(), re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    return re.findall(r"(\w+)\s*;", body)


@pytest.fixture(scope="module")
def lib(engine_lib):
    return engine_lib


def test_library_exports_every_declared_symbol(lib):
    decl = declared_functions()
    assert decl == sorted(["orx_abi_version", "orx_last_error", "orx_validate_cfg", "orx_reset",
                           "orx_step", "orx_step_events", "orx_policy", "orx_rollout",
                           "orx_dungeon_stairs", "orx_dungeon_spawn", "orx_seed_mt",
                           "orx_build_id", "orx_rollout_lanes", "orx_dstore_depths",
                           "orx_rollout_shape", "orx_rollout_concurrent", "orx_env_step",
                           "orx_rollout_ex", "orx_env_step_ex", "orx_step_n", "orx_max_events",
                           "orx_step_n_ex", "orx_env_step_args"])
    from optimax_rogue_amd import _lib
    assert sorted(_lib.EXPORTS) == decl
    for name in decl:
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "optimax_rogue_amd",
                                                                     "liborx.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (orx_\w+)", out))
    assert set(decl) <= exported


def test_library_is_built_from_the_tree(lib):
    """orx_build_id() is the hash of the tree's own orx_engine.hip + orx.h."""
    from optimax_rogue_amd import _lib, build
    assert _lib.build_id() == build.source_id()


def test_diagnostic_builds_carry_their_defines_in_the_build_id():
    """A -DORX_DIAG / -DORX_STAMPS library (build.VARIANTS, built by the
    committed recipe) reports an id that differs from the product's, so it can
    never pass test_library_is_built_from_the_tree."""
    from optimax_rogue_amd import build
    prod = build.source_id()
    ids = {v: build.source_id(d) for v, d in build.VARIANTS.items()}
    assert len(set(ids.values()) | {prod}) == len(ids) + 1
    for v, i in ids.items():
        assert i.startswith(prod + "+") and all(d in i for d in build.VARIANTS[v])
    assert build.source_id(["B=1", "A=2"]) == build.source_id(["A=2", "B=1"])


def test_build_cli_routes_variants(monkeypatch, tmp_path):
    """`--variant NAME [--out PATH]` builds that variant's -D set (into PATH
    when given), never the product build (the compile itself is stubbed)."""
    from optimax_rogue_amd import build
    calls = []
    monkeypatch.setattr(build, "build", lambda force, verbose=False, defines=(), out=None:
                        calls.append((tuple(defines), out)) or str(out))
    out = str(tmp_path / "d16.so")
    build.main(["--variant", "diag16", "--out", out])
    assert calls == [(("ORX_DIAG=16",), out)]
    calls.clear()
    build.main(["--variant", "diag32", "--define", "ORX_STREAM_AUX=0"])
    assert calls == [(("ORX_DIAG=32", "ORX_STREAM_AUX=0"),
                      os.path.join(build.AB_LIBS, "diag32.so"))]
    calls.clear()
    build.main(["--define", "ORX_DIAG=96", "--out", out])
    assert calls == [(("ORX_DIAG=96",), out)]
    with pytest.raises(SystemExit):
        build.main(["--variant", "diag16", "--variant", "diag32", "--out", out])


def test_struct_layouts_match_header():
    from optimax_rogue_amd._lib import OrxState
    from optimax_rogue_amd.config import CFG_FIELDS, OrxCfg
    from oracle.oracle import CFG_FIELDS as ORACLE_FIELDS
    assert list(CFG_FIELDS) == struct_fields("orx_cfg") == list(ORACLE_FIELDS)
    assert [f for f, _ in OrxState._fields_] == struct_fields("orx_state")
    from optimax_rogue_amd._lib import OrxRolloutShape
    assert [f for f, _ in OrxRolloutShape._fields_] == struct_fields("orx_rollout_shape")
    assert ctypes.sizeof(OrxCfg) == 4 * len(CFG_FIELDS)
    assert ctypes.sizeof(OrxState) == 8 * len(OrxState._fields_)


def test_enum_values_match_header():
    from optimax_rogue_amd import enums
    t = header_text()
    val = lambda n: int(re.search(r"#define %s (-?\d+)" % n, t).group(1))
    assert [m.value for m in enums.Move] == [val("ORX_MOVE_UP"), val("ORX_MOVE_RIGHT"),
                                             val("ORX_MOVE_DOWN"), val("ORX_MOVE_LEFT"),
                                             val("ORX_MOVE_STAY")]
    assert [r.value for r in enums.UpdateResult] == [val("ORX_IN_PROGRESS"), val("ORX_PLAYER1_WIN"),
                                                     val("ORX_PLAYER2_WIN"), val("ORX_TIE")]
    assert enums.STATUS_BAD_ACTION == val("ORX_STATUS_BAD_ACTION")
    assert enums.MAX_NPCS == val("ORX_MAX_NPCS")
    assert len(enums.OBS_FIELDS) == val("ORX_OBS_FIELDS")
    assert (enums.EV_COMBAT, enums.EV_DEATH, enums.EV_POSITION, enums.EV_DUNGEON) == (
        val("ORX_EV_COMBAT"), val("ORX_EV_DEATH"), val("ORX_EV_POSITION"), val("ORX_EV_DUNGEON"))
    assert enums.MAX_EVENTS == val("ORX_MAX_EVENTS")
    assert enums.SEP_PERIOD_MAX == val("ORX_SEP_PERIOD_MAX")
    assert [p.value for p in enums.NpcPolicy] == [val("ORX_NPC_STAY"), val("ORX_NPC_RANDOM"),
                                                  val("ORX_NPC_CHASE")]


def test_validate_cfg(lib):
    from optimax_rogue_amd import EnvConfig
    ok = [EnvConfig.c1(), EnvConfig.c3(), EnvConfig.c5(), EnvConfig(width=4, height=4),
          EnvConfig(n_npcs=17), EnvConfig(n_npcs=255, width=20, height=20),
          EnvConfig(start_mode=2, p1_depth=0, p2_depth=1000, n_npcs=16, width=40, height=10)]
    bad = [EnvConfig(width=3), EnvConfig(despawn=3), EnvConfig(start_mode=2, p1_depth=5,
                                                                p2_depth=5),
           EnvConfig(n_npcs=256), EnvConfig(n_npcs=2, width=300), EnvConfig(max_ticks=-1),
           EnvConfig(n_npcs=17, flags=32),
           EnvConfig(width=4, height=4, n_npcs=2), EnvConfig(flags=1),
           EnvConfig(n_npcs=1, npc_health=0)]
    # dungeon bank: n_layouts rides in the struct (the layouts themselves are
    # validated by DungeonBank on the host)
    import numpy as np
    lay = np.ones((2, 300, 300), np.uint8)
    bad.append(EnvConfig(width=300, height=300, layouts=lay))          # W*H > 65536
    ok.append(EnvConfig(width=6, height=5, layouts=np.ones((3, 6, 5), np.uint8)))
    # build extensions: known bits only; separation damage needs a period
    ok.append(EnvConfig(flags=3, sep_period=5))
    ok.append(EnvConfig(flags=1, sep_period=1 << 24))
    bad += [EnvConfig(flags=1, sep_period=0), EnvConfig(flags=1, sep_period=(1 << 24) + 1)]
    # the readme's character mechanics: heal needs mana; every parameter in range
    ok += [EnvConfig(flags=4 | 8 | 16 | 32, n_npcs=4), EnvConfig(flags=16, xp_per_kill=0)]
    ok.append(EnvConfig(flags=64))
    bad += [EnvConfig(flags=128), EnvConfig(flags=64, combat_cooldown=-1)]
    bad += [EnvConfig(flags=8), EnvConfig(flags=4, mana_max=2), EnvConfig(flags=4, mana_per_point=0),
            EnvConfig(flags=4, mana_regen=-1), EnvConfig(flags=16, xp_per_level=0),
            EnvConfig(flags=32, item_drop_pct=101), EnvConfig(flags=32, item_slots=-1)]
    # stock-seed word source (MT19937): staircases pack 8+8 bits
    ok.append(EnvConfig(rng=1, n_npcs=3))
    bad += [EnvConfig(rng=2), EnvConfig(rng=1, width=300, height=8)]
    # moving NPCs (the enemy AI): known policies, with the separation and
    # double-death extensions only
    ok += [EnvConfig(n_npcs=8, npc_policy=1), EnvConfig(n_npcs=40, npc_policy=2),
           EnvConfig(npc_policy=1), EnvConfig(n_npcs=3, npc_policy=2, rng=1),
           EnvConfig(n_npcs=3, npc_policy=1, flags=3, sep_period=4)]
    bad += [EnvConfig(n_npcs=8, npc_policy=3), EnvConfig(n_npcs=8, npc_policy=-1),
            EnvConfig(n_npcs=8, npc_policy=1, flags=4), EnvConfig(n_npcs=8, npc_policy=2,
                                                                   flags=64)]
    for c in ok:
        assert lib.orx_validate_cfg(ctypes.byref(c.to_c())) == 0, c
    for c in bad:
        assert lib.orx_validate_cfg(ctypes.byref(c.to_c())) == -22, c
        assert lib.orx_last_error()


def test_max_events(lib):
    """orx_max_events: ORX_MAX_EVENTS with Stay NPCs, 6 + 2 K records per game
    when the NPCs move (each NPC's own move, combat or staircase death plus
    its sweep; the players' moves, descends and health changes)."""
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.enums import MAX_EVENTS
    n = lambda c: lib.orx_max_events(ctypes.byref(c.to_c()))
    assert n(EnvConfig(n_npcs=255)) == MAX_EVENTS
    assert n(EnvConfig(n_npcs=1, npc_policy=1)) == MAX_EVENTS
    assert n(EnvConfig(n_npcs=8, npc_policy=1)) == 22
    assert n(EnvConfig(n_npcs=255, width=20, height=20, npc_policy=2)) == 516
    assert n(EnvConfig(n_npcs=8, npc_policy=7)) == -22


def test_plain_c_consumer(lib, tmp_path):
    exe = tmp_path / "abi_check"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "abi_check.c"), "-o", str(exe),
                    "-L", os.path.join(ROOT, "optimax_rogue_amd"), "-lorx",
                    "-Wl,-rpath," + os.path.join(ROOT, "optimax_rogue_amd")], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sizeof(orx_cfg_t)=116" in r.stdout
    # the ctypes mirror of orx_env_step_args_t matches the C layout
    from optimax_rogue_amd._lib import OrxEnvStepArgs
    assert f"sizeof(orx_env_step_args_t)={ctypes.sizeof(OrxEnvStepArgs)}" in r.stdout
    assert f"off_stream={OrxEnvStepArgs.stream.offset}" in r.stdout


def test_engine_refuses_cpu():
    import torch
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd.engine import BatchedEngine
    with pytest.raises(RuntimeError):
        BatchedEngine(EnvConfig(), 8, device=torch.device("cpu"))


def test_rollout_shape_rules(lib):
    """orx_rollout_shape (no device work; 1,024 SIMDs assumed without a GPU):
    the paired two-lanes-per-game form for RandomBot / StaircaseBot
    trajectory launches without dense NPCs (K <= 16, register slots) below 64
    games per wave (counting the launches that share the device; the bench's
    C3 shards: pair_rollout_kernel<8, 1, 2, false>), nontemporal stores only
    for whole-line row segments (32+ games per wave)."""
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd._lib import OrxRolloutShape

    def shape(cfg, B, p1=1, p2=1, traj=1, conc=1, n_layouts=0):
        out = OrxRolloutShape()
        c = cfg.to_c()
        c.n_layouts = n_layouts
        assert lib.orx_rollout_shape(ctypes.byref(c), p1, p2, B, traj, conc,
                                     ctypes.byref(out)) == 0
        return out.games_per_wave, out.lanes_per_game, out.nontemporal

    assert shape(EnvConfig.c5(), 16384, 2, 2) == (8, 2, 0)       # C5's 8-GPU share
    assert shape(EnvConfig.c2(), 4096) == (8, 2, 0)               # C2
    assert shape(EnvConfig.c5(), 32768, 2, 2) == (16, 2, 0)
    assert shape(EnvConfig.c5(), 131072, 2, 2) == (64, 1, 1)      # full waves: one lane per game
    assert shape(EnvConfig.c3(), 32768, conc=2) == (32, 2, 1)     # the bench's two stream shards
    assert shape(EnvConfig.c3(), 32768) == (16, 2, 0)             # one such launch alone
    assert shape(EnvConfig.c3(), 65536) == (64, 1, 1)             # full waves: one lane per game
    assert shape(EnvConfig(n_npcs=40), 4096) == (16, 1, 0)        # LDS NPC table: one lane per game
    # round 5: a RandomBot against a StaircaseBot pairs too (PM 4 / 5), not
    # with extension flags or a dungeon bank (the generic one-lane form)
    assert shape(EnvConfig.c5(), 16384, 2, 1) == (8, 2, 0)
    assert shape(EnvConfig.c3(), 32768, 1, 2, conc=2) == (32, 2, 1)
    assert shape(EnvConfig(width=20, height=20, flags=1, sep_period=3), 4096, 1, 2) == (16, 1, 1)
    assert shape(EnvConfig(width=12, height=10), 4096, 2, 1, n_layouts=4)[1] == 1
    assert shape(EnvConfig.c3(), 65536, 1, 2) == (64, 1, 1)       # full waves: one lane
    assert shape(EnvConfig.c2(), 4096, traj=0) == (16, 1, 1)      # no trajectory buffers
    # round 4: the character mechanics and dungeon banks pair too (a bank not
    # with separation damage for StaircaseBots)
    rpg = EnvConfig(width=64, height=64, n_npcs=8, flags=4 | 8 | 16 | 32)
    assert shape(rpg, 32768, conc=2) == (32, 2, 1)
    assert shape(rpg, 4096) == (8, 2, 0)
    assert shape(EnvConfig.c3(), 32768, conc=2, n_layouts=16) == (32, 2, 1)
    assert shape(EnvConfig(width=12, height=10), 4096, 2, 2, n_layouts=4) == (8, 2, 0)
    assert shape(EnvConfig(width=12, height=10, flags=1, sep_period=2), 4096, 2, 2,
                 n_layouts=4)[1] == 1
    assert shape(EnvConfig(width=300, height=200), 4096, 2, 2)[1] == 1  # packed cells: <= 256
    # round 5: C5's 131,072 games on one GPU as two 65,536-game stream shards
    # pair at 32 games per wave (StaircaseBots; one launch stays one-lane)
    assert shape(EnvConfig.c5(), 65536, 2, 2, conc=2) == (32, 2, 1)
    assert shape(EnvConfig.c5(), 131072, 2, 2, conc=2)[1] == 1     # 8 waves per SIMD: no
    assert shape(EnvConfig.c3(), 65536, conc=2) == (64, 1, 1)       # RandomBots: not measured
    bad = OrxRolloutShape()
    assert lib.orx_rollout_shape(ctypes.byref(EnvConfig.c2().to_c()), 9, 1, 64, 1, 1,
                                 ctypes.byref(bad)) == -22
    assert lib.orx_rollout_shape(ctypes.byref(EnvConfig.c2().to_c()), 1, 1, 64, 1, 0,
                                 ctypes.byref(bad)) == -22


def test_rollout_shape_bank_lds(lib, monkeypatch):
    """Round 5: a dungeon bank stays paired with its tiles in LDS up to the
    device's per-workgroup limit (160 KiB on gfx950, assumed here without a
    GPU); above half of it the paired workgroup is 512 threads (one per CU,
    two waves per SIMD); a larger bank, or a refused limit raise
    (ORX_REFUSE_LDS_RAISE=1), takes the one-lane form with its tiles in
    global memory -- never a paired launch without them."""
    from optimax_rogue_amd import EnvConfig
    from optimax_rogue_amd._lib import OrxRolloutShape

    def shape(n_layouts, B=32768, conc=2):
        out = OrxRolloutShape()
        c = EnvConfig.c3().to_c()
        c.n_layouts = n_layouts
        assert lib.orx_rollout_shape(ctypes.byref(c), 1, 1, B, 1, conc, ctypes.byref(out)) == 0
        return (out.games_per_wave, out.lanes_per_game, out.threads_per_block, out.lds_bytes)

    assert shape(16) == (32, 2, 256, 65536)        # the bench's bank: exactly 64 KiB
    assert shape(20) == (32, 2, 256, 81920)        # two workgroups per CU still fit
    assert shape(24) == (32, 2, 512, 98304)        # one per CU: 512 threads
    assert shape(40) == (32, 2, 512, 163840)       # the whole 160 KiB
    assert shape(41)[1:] == (1, 256, 0)            # too large: one lane, global tiles
    monkeypatch.setenv("ORX_REFUSE_LDS_RAISE", "1")
    assert shape(16) == (32, 2, 256, 65536)        # no raise needed
    assert shape(24)[1:] == (1, 256, 0)            # refused: one lane, global tiles
    monkeypatch.delenv("ORX_REFUSE_LDS_RAISE")
    monkeypatch.setenv("ORX_ROLLOUT_THREADS", "256")
    assert shape(24) == (32, 2, 256, 98304)        # the override (measurements)
