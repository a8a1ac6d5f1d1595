"""ctypes loader for liborx.so (the HIP engine, C-ABI in include/orx.h).

There is no fallback: if the library is missing or cannot be loaded, every
engine call raises.  Build it with ``python -m optimax_rogue_amd.build`` (or
``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os

from .config import OrxCfg

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "liborx.so")
ABI_VERSION = 7


class OrxState(ctypes.Structure):
    """ctypes mirror of orx_state_t (device pointers)."""
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "p_x", "p_y", "p_depth", "p_health", "st_x", "st_y", "tick", "status", "episode",
        "ret_sum", "ep_count", "counters", "npc_pos", "npc_health", "npc_alive",
        "p_layout", "bank_tiles", "bank_ground", "bank_meta", "sep_start", "mt_py", "mt_np",
        "dstore", "p_rpg", "item_pos", "item_mask", "npc_grid")]


class OrxRolloutShape(ctypes.Structure):
    """ctypes mirror of orx_rollout_shape_t."""
    _fields_ = [(n, ctypes.c_int32) for n in ("games_per_wave", "lanes_per_game", "nontemporal",
                                                "threads_per_block", "lds_bytes")]


class OrxEnvStepArgs(ctypes.Structure):
    """ctypes mirror of orx_env_step_args_t (orx_env_step_ex's arguments in
    one block: VecEnv.step updates a prebuilt block and passes one pointer)."""
    _fields_ = [("cfg", ctypes.POINTER(OrxCfg)), ("st", ctypes.POINTER(OrxState)),
                ("actions", ctypes.c_void_p), ("action_bytes", ctypes.c_int32),
                ("action_cols", ctypes.c_int32), ("policy_p2", ctypes.c_int32),
                ("pad0", ctypes.c_int32), ("act", ctypes.c_void_p), ("obs", ctypes.c_void_p),
                ("reward", ctypes.c_void_p), ("done", ctypes.c_void_p),
                ("status", ctypes.c_void_p), ("bad_actions", ctypes.c_void_p),
                ("n_games", ctypes.c_int64), ("seed", ctypes.c_uint64),
                ("game_offset", ctypes.c_int64), ("stream", ctypes.c_void_p)]


class OrxError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} returned {code}: {msg}")
        self.code = code


_lib = None

EXPORTS = ("orx_abi_version", "orx_last_error", "orx_validate_cfg", "orx_reset", "orx_step",
           "orx_step_events", "orx_policy", "orx_rollout", "orx_dungeon_stairs",
           "orx_dungeon_spawn", "orx_seed_mt", "orx_build_id", "orx_rollout_lanes", "orx_dstore_depths",
           "orx_rollout_shape", "orx_rollout_concurrent", "orx_env_step",
           "orx_rollout_ex", "orx_env_step_ex", "orx_step_n", "orx_max_events",
           "orx_step_n_ex", "orx_env_step_args")


def load() -> ctypes.CDLL:
    """Loads liborx.so once.  torch is imported first so the library binds to the
    HIP runtime (libamdhip64.so.7) already mapped by PyTorch-ROCm."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (HIP runtime first)
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"HIP engine library missing: {LIB_PATH} -- run "
                           "`python -m optimax_rogue_amd.build` first")
    L = ctypes.CDLL(LIB_PATH)
    vp, i64, i32, u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64
    P = ctypes.POINTER
    L.orx_abi_version.restype = ctypes.c_int
    L.orx_abi_version.argtypes = []
    L.orx_last_error.restype = ctypes.c_char_p
    L.orx_last_error.argtypes = []
    L.orx_validate_cfg.restype = ctypes.c_int
    L.orx_validate_cfg.argtypes = [P(OrxCfg)]
    L.orx_reset.restype = ctypes.c_int
    L.orx_reset.argtypes = [P(OrxCfg), P(OrxState), vp, i64, u64, i64, vp]
    L.orx_step.restype = ctypes.c_int
    L.orx_step.argtypes = [P(OrxCfg), P(OrxState), vp, i64, u64, i64, vp]
    L.orx_step_events.restype = ctypes.c_int
    L.orx_step_events.argtypes = [P(OrxCfg), P(OrxState), vp, vp, vp, i64, u64, i64, vp]
    L.orx_policy.restype = ctypes.c_int
    L.orx_policy.argtypes = [P(OrxCfg), P(OrxState), i32, i32, vp, i64, u64, i64, vp]
    L.orx_rollout.restype = ctypes.c_int
    L.orx_rollout.argtypes = [P(OrxCfg), P(OrxState), i32, i32, i32, vp, vp, i64, u64, i64, vp]
    L.orx_dungeon_stairs.restype = ctypes.c_int
    L.orx_dungeon_stairs.argtypes = [P(OrxCfg), vp, vp, vp, vp, vp, vp, i64, u64, vp]
    L.orx_dungeon_spawn.restype = ctypes.c_int
    L.orx_dungeon_spawn.argtypes = [P(OrxCfg), P(OrxState), vp, vp, vp, vp, vp, vp, vp, i64, u64,
                                    vp]
    L.orx_seed_mt.restype = ctypes.c_int
    L.orx_seed_mt.argtypes = [P(OrxCfg), P(OrxState), i64, u64, i64, vp]
    L.orx_build_id.restype = ctypes.c_char_p
    L.orx_build_id.argtypes = []
    L.orx_rollout_lanes.restype = ctypes.c_int
    L.orx_rollout_lanes.argtypes = [i64]
    # (bound only when present: an A/B diagnostic may load an older build)
    if hasattr(L, "orx_rollout_shape"):
        L.orx_rollout_shape.restype = ctypes.c_int
        L.orx_rollout_shape.argtypes = [P(OrxCfg), i32, i32, i64, i32, i32, P(OrxRolloutShape)]
    if hasattr(L, "orx_rollout_concurrent"):
        L.orx_rollout_concurrent.restype = ctypes.c_int
        L.orx_rollout_concurrent.argtypes = [P(OrxCfg), P(OrxState), i32, i32, i32, vp, vp, i64,
                                             u64, i64, i32, vp]
    if hasattr(L, "orx_rollout_ex"):
        L.orx_rollout_ex.restype = ctypes.c_int
        L.orx_rollout_ex.argtypes = [P(OrxCfg), P(OrxState), i32, i32, i32, vp, vp, i32, i64, u64,
                                     i64, i32, vp]
    if hasattr(L, "orx_env_step"):
        L.orx_env_step.restype = ctypes.c_int
        L.orx_env_step.argtypes = [P(OrxCfg), P(OrxState), vp, i32, i32, i32, vp, vp, vp, vp, vp,
                                   i64, u64, i64, vp]
    if hasattr(L, "orx_env_step_ex"):
        L.orx_env_step_ex.restype = ctypes.c_int
        L.orx_env_step_ex.argtypes = [P(OrxCfg), P(OrxState), vp, i32, i32, i32, vp, vp, vp, vp,
                                      vp, vp, i64, u64, i64, vp]
    if hasattr(L, "orx_env_step_args"):
        L.orx_env_step_args.restype = ctypes.c_int
        L.orx_env_step_args.argtypes = [P(OrxEnvStepArgs)]
    if hasattr(L, "orx_step_n"):
        L.orx_step_n.restype = ctypes.c_int
        L.orx_step_n.argtypes = [P(OrxCfg), P(OrxState), vp, i32, vp, i32, i64, u64, i64, vp]
    if hasattr(L, "orx_step_n_ex"):
        L.orx_step_n_ex.restype = ctypes.c_int
        L.orx_step_n_ex.argtypes = [P(OrxCfg), P(OrxState), vp, i32, vp, i32, i64, u64, i64, i32,
                                    vp]
    if hasattr(L, "orx_max_events"):
        L.orx_max_events.restype = ctypes.c_int
        L.orx_max_events.argtypes = [P(OrxCfg)]
    if hasattr(L, "orx_dstore_depths"):
        L.orx_dstore_depths.restype = ctypes.c_int
        L.orx_dstore_depths.argtypes = [P(OrxCfg)]
    v = L.orx_abi_version()
    if v != ABI_VERSION:
        raise RuntimeError(f"liborx.so ABI {v} != expected {ABI_VERSION}")
    _lib = L
    return L


def check(fn: str, code: int) -> None:
    if code != 0:
        msg = load().orx_last_error().decode(errors="replace")
        raise OrxError(fn, code, msg)


def build_id() -> str:
    """orx_build_id() of the loaded library (build.source_id() of its sources)."""
    return load().orx_build_id().decode()
