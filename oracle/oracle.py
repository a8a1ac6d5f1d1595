"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the C oracle (orx_oracle.c).

The oracle is the CPU restatement of the reference updater used to check the
HIP engine.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import this module; the product package never does.

Build: ``make -C oracle`` (or __graft_entry__.build()) -> oracle/liborx_oracle.so
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liborx_oracle.so")

# Field order of orx_cfg_t (include/orx.h); tests check it against the header.
CFG_FIELDS = ["width", "height", "despawn", "max_ticks", "start_mode", "p1_depth", "p2_depth",
              "n_npcs", "npc_health", "npc_damage", "npc_armor", "player_health",
              "player_damage", "player_armor", "autoreset", "flags", "n_layouts", "sep_period",
              "rng", "mana_max", "mana_regen", "mana_per_point", "xp_per_kill", "xp_per_level",
              "item_drop_pct", "item_bonus", "item_slots", "combat_cooldown", "npc_policy"]


class _Cfg(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int32) for f in CFG_FIELDS]


DEFAULT_CFG = dict(width=32, height=32, despawn=1, max_ticks=1000, start_mode=1, p1_depth=0,
                   p2_depth=0, n_npcs=0, npc_health=3, npc_damage=1, npc_armor=0,
                   player_health=10, player_damage=2, player_armor=1, autoreset=1, flags=0,
                   n_layouts=0, sep_period=0, rng=0, mana_max=9, mana_regen=1, mana_per_point=1,
                   xp_per_kill=1, xp_per_level=3, item_drop_pct=50, item_bonus=1, item_slots=3,
                   combat_cooldown=3, npc_policy=0)

_lib = None


def build(force: bool = False) -> str:
    """Compiles liborx_oracle.so with gcc (seconds)."""
    src = os.path.join(HERE, "orx_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        import subprocess
        tmp = f"{LIB_PATH}.{os.getpid()}.tmp"   # (parallel test workers: atomic replace)
        subprocess.check_call(["gcc", "-O2", "-std=c11", "-Wall", "-shared", "-fPIC", "-o",
                               tmp, src])
        os.replace(tmp, LIB_PATH)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i64, i32, u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64
        L.oracle_new.restype = vp
        L.oracle_new.argtypes = [ctypes.POINTER(_Cfg), i64, u64, i64, ctypes.c_int]
        L.oracle_free.argtypes = [vp]
        L.oracle_reset.argtypes = [vp, vp, vp]
        L.oracle_step.argtypes = [vp, vp]
        L.oracle_policy.argtypes = [vp, i32, i32, vp]
        L.oracle_export.argtypes = [vp] + [vp] * 15
        for fn in ("oracle_world", "oracle_events", "oracle_entities"):
            getattr(L, fn).argtypes = [vp, i64, vp, i32]
            getattr(L, fn).restype = i32
        L.oracle_philox.argtypes = [vp, vp, vp]
        L.oracle_set_game.argtypes = [vp, i64, vp, i32, i32, i32]
        L.oracle_rollout.argtypes = [vp, i32, i32, i32, vp]
        L.oracle_set_rng.argtypes = [vp, u64, i64]
        L.oracle_set_bank.argtypes = [vp, vp, i32]
        L.oracle_export_layout.argtypes = [vp, vp]
        L.oracle_export_sep.argtypes = [vp, vp]
        L.oracle_seed_mt.argtypes = [vp, u64]
        L.oracle_export_rpg.argtypes = [vp, vp, vp, vp]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def philox(ctr, key):
    c = np.array(ctr, np.uint32)
    k = np.array(key, np.uint32)
    out = np.zeros(4, np.uint32)
    lib().oracle_philox(_ptr(c), _ptr(k), _ptr(out))
    return tuple(int(v) for v in out)


class Oracle:
    """B reference games on the CPU (same stream keys as the engine)."""

    def __init__(self, cfg: dict, n_games: int, seed: int, game_offset: int = 0,
                 record_events: bool = False, layouts=None):
        """layouts: optional [L, W, H] Tile codes -- an explicit-grid dungeon
        generator (spawn_dungeon picks randint(L)); None = EmptyDungeonGenerator."""
        full = dict(DEFAULT_CFG)
        full.update({k: v for k, v in cfg.items() if k in CFG_FIELDS})
        full["n_layouts"] = 0 if layouts is None else len(layouts)
        self.cfg = full
        self.B = int(n_games)
        self.K = int(full["n_npcs"])
        self._c = _Cfg(**full)
        self._h = lib().oracle_new(ctypes.byref(self._c), self.B, int(seed), int(game_offset),
                                   int(record_events))
        if full["rng"] == 1:   # stock-seed mode: random.seed / np.random.seed(seed + gid)
            lib().oracle_seed_mt(self._h, int(seed))
        self.layouts = None
        if layouts is not None:
            self.layouts = np.ascontiguousarray(layouts, np.uint8)
            assert self.layouts.shape[1:] == (full["width"], full["height"])
            lib().oracle_set_bank(self._h, _ptr(self.layouts), len(self.layouts))

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                lib().oracle_free(self._h)
            except Exception:  # interpreter shutdown: the module's globals are gone
                pass
            self._h = None

    def reset(self, mask=None, episode=None):
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        e = None if episode is None else np.ascontiguousarray(episode, np.int32)
        lib().oracle_reset(self._h, None if m is None else _ptr(m), None if e is None else _ptr(e))

    def step(self, actions):
        a = np.ascontiguousarray(actions, np.int8).reshape(self.B, 2)
        lib().oracle_step(self._h, _ptr(a))

    def policy(self, pol1: int, pol2: int, actions=None):
        a = (np.full((self.B, 2), 5, np.int8) if actions is None
             else np.ascontiguousarray(actions, np.int8).reshape(self.B, 2).copy())
        lib().oracle_policy(self._h, int(pol1), int(pol2), _ptr(a))
        return a

    def set_game(self, g: int, ents, stairs):
        """Test hook: game g becomes a hand-built depth-0 state (entities
        [n][5] {iden, depth, x, y, health}, staircase (sx, sy)) at tick 1."""
        e = np.ascontiguousarray(np.asarray(ents, np.int32).reshape(-1, 5))
        lib().oracle_set_game(self._h, g, _ptr(e), len(e), int(stairs[0]), int(stairs[1]))

    def rollout(self, pol1: int, pol2: int, n_ticks: int):
        scratch = np.full((self.B, 2), 5, np.int8)
        lib().oracle_rollout(self._h, int(pol1), int(pol2), int(n_ticks), _ptr(scratch))

    def export(self) -> dict:
        B, K = self.B, self.K
        out = {k: np.zeros((2, B), np.int32) for k in
               ("p_x", "p_y", "p_depth", "p_health", "st_x", "st_y")}
        for k in ("tick", "status", "episode", "ret_sum", "ep_count"):
            out[k] = np.zeros(B, np.int32)
        out["counters"] = np.zeros((4, B), np.int32)
        out["npc_pos"] = np.zeros((K, B), np.uint16)
        out["npc_health"] = np.zeros((K, B), np.int8)
        out["npc_alive"] = np.zeros(B if K <= 32 else ((K + 31) // 32, B), np.uint32)
        order = ["p_x", "p_y", "p_depth", "p_health", "st_x", "st_y", "tick", "status",
                 "episode", "ret_sum", "ep_count", "counters", "npc_pos", "npc_health",
                 "npc_alive"]
        lib().oracle_export(self._h, *[_ptr(out[k]) for k in order])
        if self.cfg["flags"] & 1:   # ORX_EXT_SEPARATION_DAMAGE
            out["sep_start"] = np.zeros(B, np.int32)
            lib().oracle_export_sep(self._h, _ptr(out["sep_start"]))
        if self.layouts is not None:
            out["p_layout"] = np.zeros((2, B), np.int16)
            lib().oracle_export_layout(self._h, _ptr(out["p_layout"]))
        if self.cfg["flags"] & 124:  # ORX_EXT_CHARACTER: player attributes, items
            out["p_rpg"] = np.zeros((6, 2, B), np.int32)
            items = self.cfg["flags"] & 32 and K > 0
            if items:
                out["item_pos"] = np.zeros((K, B), np.uint16)
                out["item_mask"] = np.zeros((2, B), np.uint32)
            lib().oracle_export_rpg(self._h, _ptr(out["p_rpg"]),
                                    _ptr(out["item_pos"]) if items else None,
                                    _ptr(out["item_mask"]) if items else None)
        return out

    def world(self, g: int):
        """World.dungeons as (depth, sx, sy) -- plus the layout index with a bank."""
        buf = np.zeros((4096, 4), np.int32)
        n = lib().oracle_world(self._h, g, _ptr(buf), 4096)
        w = 4 if self.layouts is not None else 3
        return [tuple(int(v) for v in r[:w]) for r in buf[:n]]

    def events(self, g: int):
        buf = np.zeros((256, 4), np.int32)
        n = lib().oracle_events(self._h, g, _ptr(buf), 256)
        return [tuple(int(v) for v in r) for r in buf[:n]]

    def entities(self, g: int):
        cap = 2 + 255 + 1   # both players and up to 255 NPCs (ORX_MAX_NPCS)
        buf = np.zeros((cap, 7), np.int32)
        n = lib().oracle_entities(self._h, g, _ptr(buf), cap)
        return [tuple(int(v) for v in r) for r in buf[:n]]
