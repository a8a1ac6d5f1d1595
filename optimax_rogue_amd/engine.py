"""BatchedEngine: B independent Optimax Rogue games resident on one GPU.

PyTorch-ROCm owns every buffer (struct-of-arrays int tensors, batch axis
contiguous); the HIP kernels in liborx.so are reached through the C-ABI of
include/orx.h and run asynchronously on the current torch stream.

Reference counterpart: one ``GameState`` (optimax_rogue/game/state.py:14-34)
plus one ``Updater`` (optimax_rogue/logic/updater.py:52-69) per game.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np
import torch

from . import _lib
from .config import EnvConfig
from .enums import (EXT_CHARACTER, EXT_ITEMS, EXT_SEPARATION_DAMAGE,
                    MAX_REG_NPCS, N_COUNTERS, OBS_COMPACT, OBS_COMPACT_FIELDS, OBS_FIELDS,
                    OBS_INT32, RNG_MT19937, RPG_FIELDS, Policy)


def obs_rows(obs_format: int = OBS_INT32) -> int:
    """Rows per tick of a trajectory in ``obs_format`` (14 int32 or 6 compact)."""
    if obs_format not in (OBS_INT32, OBS_COMPACT):
        raise ValueError(f"unknown obs_format {obs_format}")
    return len(OBS_FIELDS) if obs_format == OBS_INT32 else len(OBS_COMPACT_FIELDS)


def decode_compact(obs: torch.Tensor) -> torch.Tensor:
    """ORX_OBS_COMPACT rows [T, 6, B] (int32 storage of the uint32 words) ->
    the int32 rows [T, 14, B] of OBS_FIELDS, on the rows' device."""
    w = obs.to(torch.int64) & 0xFFFFFFFF
    cells, stairs, hp, d1, d2, ts = (w[:, k] for k in range(6))
    byte = lambda v, k: (v >> (8 * k)) & 0xFF
    h16 = lambda v: ((v & 0xFFFF) ^ 0x8000) - 0x8000
    out = torch.stack([byte(cells, 0), byte(cells, 1), obs[:, 3].to(torch.int64), h16(hp),
                       byte(cells, 2), byte(cells, 3), obs[:, 4].to(torch.int64), h16(hp >> 16),
                       ts & ((1 << 27) - 1), ts >> 27, byte(stairs, 0), byte(stairs, 1),
                       byte(stairs, 2), byte(stairs, 3)], dim=1)
    return out.to(torch.int32)


STATE_FIELDS = ("p_x", "p_y", "p_depth", "p_health", "st_x", "st_y", "tick", "status", "episode",
                "ret_sum", "ep_count", "counters", "npc_pos", "npc_health", "npc_alive")
BANK_FIELDS = ("p_layout", "bank_tiles", "bank_ground", "bank_meta")


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _raw_stream_getter(device: torch.device):
    """A zero-argument callable returning the raw handle of ``device``'s current
    stream (torch's private getter when this build has it: no Stream object per
    call on the eager path)."""
    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    idx = device.index
    if raw is not None:
        return lambda: raw(idx)
    return lambda: torch.cuda.current_stream(device).cuda_stream


def cuda_device(device=None) -> torch.device:
    """``device`` with its index made explicit (``"cuda"`` / None -> the current
    device), so engines built with ``"cuda"`` and ``"cuda:0"`` compare equal and
    share the shard streams."""
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type == "cuda" and device.index is None:
        return torch.device("cuda", torch.cuda.current_device())
    return device


class BatchedEngine:
    """SoA state of ``n_games`` games and the launches that advance it.

    Global game id of local game ``i`` is ``game_offset + i``; together with
    ``seed`` and the game's episode it keys every random draw, so a game's
    trajectory does not depend on the batch it runs in (or on the GPU count).
    """

    def __init__(self, cfg: EnvConfig, n_games: int, seed: int = 0, game_offset: int = 0,
                 device: Optional[torch.device] = None, reset: bool = True):
        self.lib = _lib.load()
        self.cfg = cfg
        self._ccfg = cfg.to_c()
        code = self.lib.orx_validate_cfg(ctypes.byref(self._ccfg))
        if code != 0:
            raise ValueError(self.lib.orx_last_error().decode())
        device = cuda_device(device)
        if device.type != "cuda":
            raise RuntimeError("BatchedEngine runs on a ROCm GPU only (no CPU path)")
        self.device = device
        self.B = int(n_games)
        self.K = int(cfg.n_npcs)
        self.seed = int(seed)
        self.game_offset = int(game_offset)
        # launches sharing the device with this batch's rollouts (orx_rollout_concurrent):
        # StreamShardedEngine sets it to its stream count
        self.concurrency = 1
        B, K = self.B, self.K
        z = lambda *shape, dt=torch.int32: torch.zeros(shape, dtype=dt, device=device)
        self.p_x, self.p_y, self.p_depth, self.p_health = z(2, B), z(2, B), z(2, B), z(2, B)
        self.st_x, self.st_y = z(2, B), z(2, B)
        self.tick, self.status, self.episode = z(B), z(B), z(B)
        self.ret_sum, self.ep_count = z(B), z(B)
        self.counters = z(N_COUNTERS, B)
        # uint16 / uint32 payloads are stored in same-width signed tensors
        self.npc_pos = z(max(K, 1), B, dt=torch.int16)
        self.npc_health = z(max(K, 1), B, dt=torch.int8)
        # alive bits: [B] for K <= 32, rows of 32 above (include/orx.h)
        self.npc_alive = z(B) if K <= 32 else z((K + 31) // 32, B)
        self.actions = torch.full((B, 2), 5, dtype=torch.int8, device=device)
        ptrs = {f: getattr(self, f).data_ptr() for f in STATE_FIELDS}
        # explicit-grid dungeon generator (cfg.layouts): the bank and each
        # player's layout index; all NULL for EmptyDungeonGenerator
        self.bank = None
        if cfg.layouts is not None:
            from .dungeons import DungeonBank
            bank = DungeonBank(cfg.layouts)
            if (bank.width, bank.height) != (cfg.width, cfg.height):
                raise ValueError("layouts must be [L, width, height]")
            if bank.min_ground < K + 2:
                raise ValueError("every layout needs Ground tiles for both players and the NPCs")
            self.bank = bank
            self.p_layout = z(2, B, dt=torch.int16)
            self.bank_tiles = torch.from_numpy(bank.layouts.reshape(len(bank), -1)).to(device)
            self.bank_ground = torch.from_numpy(bank.ground.view(np.int16)).to(device)
            self.bank_meta = torch.from_numpy(bank.meta).to(device)
            ptrs.update({f: getattr(self, f).data_ptr() for f in BANK_FIELDS})
        # EXT_SEPARATION_DAMAGE state (first separated tick, -1 = together)
        self.sep_start = None
        if int(cfg.flags) & EXT_SEPARATION_DAMAGE:
            self.sep_start = torch.full((B,), -1, dtype=torch.int32, device=device)
            ptrs["sep_start"] = self.sep_start.data_ptr()
        # stock-seed mode: each game's CPython random and numpy RandomState
        # (MT19937 key words + index, column per game) and the dungeons each
        # player entered (depth, sx | sy << 8 | (layout + 1) << 16), a ring of
        # N = orx_dstore_depths(cfg) >= max_ticks per player, slot (depth -
        # the player's start depth) mod N
        self.mt_py = self.mt_np = self.dstore = None
        if int(cfg.rng) == RNG_MT19937:
            self.mt_py, self.mt_np = z(625, B), z(625, B)
            n = int(self.lib.orx_dstore_depths(ctypes.byref(self._ccfg)))
            _lib.check("orx_dstore_depths", min(n, 0))
            self._warn_dstore(n)
            self.dstore = z(2, n, 2, B)
            ptrs.update({f: getattr(self, f).data_ptr() for f in ("mt_py", "mt_np", "dstore")})
        # the readme's character mechanics (EXT_CHARACTER flags): player attributes
        # [RPG_FIELDS][2][B]; with EXT_ITEMS and NPCs the items each NPC slot
        # dropped (x | y << 8) and their on-floor / kind bit masks
        self.p_rpg = self.item_pos = self.item_mask = None
        if int(cfg.flags) & EXT_CHARACTER:
            self.p_rpg = z(len(RPG_FIELDS), 2, B)
            ptrs["p_rpg"] = self.p_rpg.data_ptr()
            if int(cfg.flags) & EXT_ITEMS and K > 0:
                self.item_pos = z(K, B, dt=torch.int16)
                self.item_mask = z(2, B)
                ptrs.update(item_pos=self.item_pos.data_ptr(), item_mask=self.item_mask.data_ptr())
        # dense NPCs (K > MAX_REG_NPCS): each game's occupancy grid of the NPC
        # depth in HBM (slot + 1 per cell; 4 KiB per 64x64 game)
        self.npc_grid = None
        if K > MAX_REG_NPCS:
            self.npc_grid = torch.zeros((B, int(cfg.width) * int(cfg.height)), dtype=torch.uint8,
                                        device=device)
            ptrs["npc_grid"] = self.npc_grid.data_ptr()
        self._st = _lib.OrxState(**ptrs)
        self._pcfg, self._pst = ctypes.byref(self._ccfg), ctypes.byref(self._st)
        if self.mt_py is not None:
            self.seed_rng()
        if reset:
            self.reset()

    # -- plumbing -----------------------------------------------------------
    def _warn_dstore(self, n_depths: int) -> int:
        """Stock-seed mode's dungeon store costs 16 * N bytes per game (N =
        orx_dstore_depths >= max_ticks; orx_seed_mt clears all of it): warns
        when the batch's store exceeds a quarter of the device's memory.
        Returns the store's bytes."""
        import warnings
        nbytes = 16 * int(n_depths) * self.B
        total = torch.cuda.get_device_properties(self.device).total_memory
        if nbytes > total // 4:
            warnings.warn(f"stock-seed dungeon store: {nbytes / 2**30:.1f} GiB for {self.B} games "
                          f"({16 * n_depths} B per game at max_ticks {self.cfg.max_ticks}), more "
                          f"than a quarter of {self.device}'s memory", RuntimeWarning)
        return nbytes

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _call(self, name, *args):
        fn = getattr(self.lib, name)
        if torch.cuda.current_device() == self.device.index:
            code = fn(self._pcfg, self._pst, *args)
        else:
            with torch.cuda.device(self.device):
                code = fn(self._pcfg, self._pst, *args)
        _lib.check(name, code)

    def rollout_launcher(self, n_ticks: int, p1: int = Policy.Random, p2: int = Policy.Random,
                         obs: Optional[torch.Tensor] = None, act: Optional[torch.Tensor] = None,
                         obs_format: int = OBS_INT32):
        """A zero-argument callable that launches ``rollout(n_ticks, p1, p2, obs,
        act, obs_format)`` on the current stream of this moment, its C
        arguments bound once (a timed loop then pays one ctypes call per
        launch, nothing else)."""
        self._check_traj(n_ticks, obs, act, obs_format)
        fn, check = self.lib.orx_rollout_ex, _lib.check
        args = (self._pcfg, self._pst, int(p1), int(p2), int(n_ticks), _ptr(obs), _ptr(act),
                int(obs_format), self.B, self.seed, self.game_offset, int(self.concurrency),
                self._stream())

        def launch():
            code = fn(*args)
            if code:
                check("orx_rollout_ex", code)
        return launch

    def rollout_lanes(self) -> int:
        """Games per wave of this batch's one-lane rollout launches
        (orx_rollout_lanes); rollout_shape() gives the launch's actual form."""
        return int(self.lib.orx_rollout_lanes(self.B))

    def rollout_shape(self, p1: int = Policy.Random, p2: int = Policy.Random,
                      trajectory: bool = True) -> dict:
        """The shape orx_rollout launches these arguments with
        (orx_rollout_shape): games per wave, lanes per game (2 = the paired
        form), nontemporal trajectory stores, threads per workgroup and
        dynamic LDS bytes per workgroup (a bank's staged tiles)."""
        out = _lib.OrxRolloutShape()
        code = self.lib.orx_rollout_shape(self._pcfg, int(p1), int(p2), self.B, int(trajectory),
                                          int(self.concurrency), ctypes.byref(out))
        _lib.check("orx_rollout_shape", code)
        return {"games_per_wave": out.games_per_wave, "lanes_per_game": out.lanes_per_game,
                "nontemporal": bool(out.nontemporal), "threads_per_block": out.threads_per_block,
                "lds_bytes": out.lds_bytes}

    # -- the C-ABI entry points -------------------------------------------
    def seed_rng(self, seed: Optional[int] = None) -> None:
        """Stock-seed mode: random.seed(n) and np.random.seed(n) for every game,
        n = seed + global game id (orx_seed_mt)."""
        if seed is not None:
            self.seed = int(seed)
        self._call("orx_seed_mt", self.B, self.seed, self.game_offset, self._stream())

    def reset(self, mask: Optional[torch.Tensor] = None, episode=None) -> None:
        """GameStartGenerator.setup_game for the masked games (all if None).

        ``episode`` (int or tensor) sets the episode index first; by default
        a full reset starts every game at episode 0."""
        if mask is not None and mask.numel() != self.B:
            raise ValueError("mask must have n_games elements")
        if mask is None and episode is None:
            episode = 0
        if episode is not None:
            ep = torch.as_tensor(episode, dtype=torch.int32, device=self.device)
            if mask is None:
                self.episode.copy_(ep.expand(self.B))
            else:
                m = mask.to(self.device).bool()
                self.episode.copy_(torch.where(m, ep.expand(self.B), self.episode))
        m8 = None
        if mask is not None:
            m8 = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        self._call("orx_reset", _ptr(m8), self.B, self.seed, self.game_offset, self._stream())

    def step(self, actions: Optional[torch.Tensor] = None, events: bool = False):
        """Updater.update for every game: actions[b] = (player 1, player 2) Move
        values.  Returns the status tensor (UpdateResult codes, asynchronous);
        with ``events=True`` returns ``(status, events, n_events)``: the tick's
        update-event records int32 [n_games, max_events(), 4] and their counts
        (include/orx.h ORX_EV_*), in the reference's GameStateUpdate order;
        both buffers belong to the engine and are overwritten by the next
        ``step(events=True)``."""
        a = self.actions if actions is None else actions
        self._check_actions(a, "actions")
        if not events:
            self._call("orx_step", _ptr(a), self.B, self.seed, self.game_offset, self._stream())
            return self.status
        if getattr(self, "_ev", None) is None:
            self._ev = torch.zeros((self.B, self.max_events(), 4), dtype=torch.int32,
                                   device=self.device)
            self._nev = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        self._call("orx_step_events", _ptr(a), _ptr(self._ev), _ptr(self._nev), self.B, self.seed,
                   self.game_offset, self._stream())
        return self.status, self._ev, self._nev

    def max_events(self) -> int:
        """Event records per game-tick of ``step(events=True)`` for this
        configuration (orx_max_events: MAX_EVENTS, or 6 + 2 K with moving
        NPCs)."""
        n = int(self.lib.orx_max_events(self._pcfg))
        _lib.check("orx_max_events", min(n, 0))
        return n

    def step_n(self, actions: torch.Tensor, obs: Optional[torch.Tensor] = None,
               obs_format: int = OBS_INT32) -> torch.Tensor:
        """orx_step_n: ``actions`` int8 [T, n_games, 2] (a move log: tick t plays
        actions[t]) stepped in one launch, exactly as T calls of ``step`` would;
        ``obs`` (int32 [T, obs_rows(obs_format), n_games], optional) receives
        every tick's observation.  Returns the status tensor."""
        if actions.dtype != torch.int8 or actions.dim() != 3 or actions.shape[1:] != (self.B, 2) \
                or not actions.is_contiguous() or actions.device != self.device:
            raise ValueError(f"actions must be a contiguous int8 [T, n_games, 2] tensor on "
                             f"{self.device}")
        T = int(actions.shape[0])
        self._check_traj(T, obs, None, obs_format)
        self._call("orx_step_n_ex", _ptr(actions), T, _ptr(obs), int(obs_format), self.B,
                   self.seed, self.game_offset, int(self.concurrency), self._stream())
        return self.status

    # learner action widths orx_env_step_ex reads (uint8 as int8: 1..6 read
    # the same, and 128..255 become negative, i.e. refused like any other
    # value outside the Move codes)
    _ACTION_BYTES = {torch.int8: 1, torch.uint8: 1, torch.int16: 2, torch.int32: 4,
                     torch.int64: 8}

    def env_step(self, actions: torch.Tensor, p2: int, obs: torch.Tensor, reward: torch.Tensor,
                 done: torch.Tensor, status: torch.Tensor,
                 bad_actions: Optional[torch.Tensor] = None) -> None:
        """orx_env_step_ex: one learner tick in one launch.  ``actions``:
        integer [n_games] (player 1; player 2 moved by policy ``p2``, not
        Policy.NONE) or [n_games, 2], any integer width, contiguous, on the
        engine's device (values outside the Move codes stop that game with
        STATUS_BAD_ACTION).  Writes the pair played into ``self.actions``,
        then obs int32 [n_games, 14], reward float32, done bool and status
        int32 [n_games]; ``bad_actions`` (int32 [1] on the device, or None)
        is incremented by the number of games whose actions were refused."""
        nb = self._ACTION_BYTES.get(actions.dtype)
        if nb is None or tuple(actions.shape) not in ((self.B,), (self.B, 2)) \
                or not actions.is_contiguous() or actions.device != self.device:
            raise ValueError(f"actions must be a contiguous integer [n_games] or [n_games, 2] "
                             f"tensor on {self.device}")
        outs = [(obs, torch.int32, (self.B, len(OBS_FIELDS))), (reward, torch.float32, (self.B,)),
                (done, torch.bool, (self.B,)), (status, torch.int32, (self.B,))]
        if bad_actions is not None:
            outs.append((bad_actions, torch.int32, (1,)))
        for t, dt, shape in outs:
            if t.dtype != dt or tuple(t.shape) != shape or not t.is_contiguous() \
                    or t.device != self.device:
                raise ValueError(f"env_step output must be a contiguous {dt} {shape} tensor")
        self._env_step_raw(actions, nb, int(p2), obs, reward, done, status, bad_actions)

    def _env_step_raw(self, actions, nb, p2, obs, reward, done, status=None,
                      bad_actions=None) -> None:
        """orx_env_step_ex on tensors already checked: one ctypes call; status
        and bad_actions may be None."""
        code = self.lib.orx_env_step_ex(
            self._pcfg, self._pst, actions.data_ptr(), nb, actions.dim(), p2,
            self.actions.data_ptr(), obs.data_ptr(), reward.data_ptr(), done.data_ptr(),
            None if status is None else status.data_ptr(),
            None if bad_actions is None else bad_actions.data_ptr(), self.B, self.seed,
            self.game_offset, torch.cuda.current_stream(self.device).cuda_stream)
        if code:
            _lib.check("orx_env_step_ex", code)

    def env_step_launcher(self, p2: int):
        """A callable ``launch(actions, nb, cols, obs, reward, done, status, bad)``
        -- orx_env_step_ex with every argument that does not change between
        ticks bound once (VecEnv.step's eager path: one ctypes call, the
        pointers as plain integers).  The caller has checked the tensors."""
        fn, check = self.lib.orx_env_step_ex, _lib.check
        pcfg, pst, act = self._pcfg, self._pst, self.actions.data_ptr()
        B, p2 = self.B, int(p2)
        stream = _raw_stream_getter(self.device)
        eng = self

        def launch(a_ptr, nb, cols, obs, rew, done, status, bad):
            # seed and game_offset read per call: a later change to the
            # engine's keys reaches this path as it reaches step / rollout
            code = fn(pcfg, pst, a_ptr, nb, cols, p2, act, obs, rew, done, status, bad, B,
                      eng.seed, eng.game_offset, stream())
            if code:
                check("orx_env_step_ex", code)
        return launch

    def env_step_slot(self, p2: int, obs: torch.Tensor, reward: torch.Tensor,
                      done: torch.Tensor, status: torch.Tensor,
                      bad_actions: Optional[torch.Tensor] = None):
        """A callable ``launch(actions_ptr, nb, cols, outs=None)`` --
        orx_env_step_args over one prebuilt argument block for this output set
        (VecEnv.step's ring of preallocated outputs: per call the actions
        pointer, the current stream and whatever changed since the last call
        are written into the block, and ctypes passes one pointer; ``outs``,
        four data pointers, redirects the block to fresh outputs).  The caller
        has checked the tensors."""
        a = _lib.OrxEnvStepArgs()
        a.cfg = ctypes.pointer(self._ccfg)
        a.st = ctypes.pointer(self._st)
        a.policy_p2 = int(p2)
        a.act = self.actions.data_ptr()
        a.obs, a.reward, a.done, a.status = (obs.data_ptr(), reward.data_ptr(), done.data_ptr(),
                                             status.data_ptr())
        a.bad_actions = None if bad_actions is None else bad_actions.data_ptr()
        a.n_games = self.B
        fn, check, ref = self.lib.orx_env_step_args, _lib.check, ctypes.byref(a)
        stream = _raw_stream_getter(self.device)
        eng = self
        last = [None, None, None, None]   # nb, cols, seed, game_offset in the block

        def launch(a_ptr, nb, cols, outs=None):
            if outs is not None:   # (fresh outputs: their four pointers this call)
                a.obs, a.reward, a.done, a.status = outs
            a.actions = a_ptr
            if nb != last[0] or cols != last[1]:
                a.action_bytes, a.action_cols = nb, cols
                last[0], last[1] = nb, cols
            # seed and game_offset read per call, as step / rollout read them
            if eng.seed != last[2] or eng.game_offset != last[3]:
                a.seed, a.game_offset = eng.seed, eng.game_offset
                last[2], last[3] = eng.seed, eng.game_offset
            a.stream = stream()
            code = fn(ref)
            if code:
                check("orx_env_step_args", code)
        launch.args = a   # (keeps the block alive with the callable)
        return launch

    def policy(self, p1: int = Policy.Random, p2: int = Policy.Random,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """RandomBot / StaircaseBot moves for both players into ``out``."""
        a = self.actions if out is None else out
        self._check_actions(a, "out")
        self._call("orx_policy", int(p1), int(p2), _ptr(a), self.B, self.seed, self.game_offset,
                   self._stream())
        return a

    def rollout(self, n_ticks: int, p1: int = Policy.Random, p2: int = Policy.Random,
                obs: Optional[torch.Tensor] = None, act: Optional[torch.Tensor] = None,
                obs_format: int = OBS_INT32) -> None:
        """n_ticks x (policy, step) fused in one launch.  ``obs`` (int32
        [n_ticks, obs_rows(obs_format), n_games]: the 14 OBS_FIELDS rows, or
        with OBS_COMPACT the 6 compact rows, decode_compact) and ``act`` (int8
        [n_ticks, n_games, 2]) receive every tick's observation and actions."""
        self._check_traj(n_ticks, obs, act, obs_format)
        self._call("orx_rollout_ex", int(p1), int(p2), int(n_ticks), _ptr(obs), _ptr(act),
                   int(obs_format), self.B, self.seed, self.game_offset, int(self.concurrency),
                   self._stream())

    def _check_actions(self, a: torch.Tensor, what: str) -> None:
        # the kernels index [n_games, 2] blindly: a wrong buffer would be an
        # out-of-bounds device access, so it is refused here
        if a.dtype != torch.int8 or tuple(a.shape) != (self.B, 2) or not a.is_contiguous() \
                or a.device != self.device:
            raise ValueError(f"{what} must be a contiguous int8 [n_games, 2] tensor on "
                             f"{self.device}")

    def _check_traj(self, n_ticks, obs, act, obs_format=OBS_INT32):
        rows = obs_rows(obs_format)
        for t, dt, n, what in ((obs, torch.int32, n_ticks * rows * self.B,
                                f"obs must be a contiguous int32 [n_ticks, {rows}, n_games] tensor"),
                               (act, torch.int8, n_ticks * self.B * 2,
                                "act must be a contiguous int8 [n_ticks, n_games, 2] tensor")):
            if t is not None and (t.dtype != dt or t.numel() < n or not t.is_contiguous()
                                  or t.device != self.device):
                raise ValueError(f"{what} on {self.device}")

    # -- host views -----------------------------------------------------------
    def snapshot(self) -> dict:
        """Copies the whole SoA state to numpy (synchronizes); with a dungeon
        bank also ``p_layout``."""
        out = {}
        if self.bank is not None:
            out["p_layout"] = self.p_layout.cpu().numpy()
        if self.sep_start is not None:
            out["sep_start"] = self.sep_start.cpu().numpy()
        if self.p_rpg is not None:
            out["p_rpg"] = self.p_rpg.cpu().numpy()
        if self.item_pos is not None:
            out["item_pos"] = self.item_pos.cpu().numpy().view(np.uint16)
            out["item_mask"] = self.item_mask.cpu().numpy().view(np.uint32)
        if self.mt_py is not None:
            for f in ("mt_py", "mt_np"):
                out[f] = getattr(self, f).cpu().numpy().view(np.uint32)
            out["dstore"] = self.dstore.cpu().numpy()
        for f in STATE_FIELDS:
            a = getattr(self, f).cpu().numpy()
            if f == "npc_pos":
                a = a.view(np.uint16)[: self.K]
            elif f == "npc_health":
                a = a[: self.K]
            elif f == "npc_alive":
                a = a.view(np.uint32)
            out[f] = a
        return out

    def _check_snapshot(self, snap: dict) -> None:
        """Refuses host state the kernels would index out of bounds with:
        players or NPCs off the grid, layout indices outside the bank."""
        W, H = int(self.cfg.width), int(self.cfg.height)

        def within(name, lo, hi, sel=None):
            if name not in snap:
                return
            a = np.asarray(snap[name]).astype(np.int64)
            if sel is not None:
                a = a[sel]
            if a.size and (a.min() < lo or a.max() >= hi):
                raise ValueError(f"snapshot {name} outside [{lo}, {hi})")
        within("p_x", 0, W)
        within("p_y", 0, H)
        within("p_depth", 0, 1 << 30)
        if self.bank is not None:
            within("p_layout", 0, len(self.bank))
        if self.K and "npc_pos" in snap:
            from .enums import npc_alive_bits
            pos = np.asarray(snap["npc_pos"]).astype(np.uint16).astype(np.int64)[: self.K]
            alive = snap.get("npc_alive")
            live = (npc_alive_bits(np.asarray(alive).astype(np.uint32), self.K)
                    if alive is not None else np.ones_like(pos, bool))
            if ((pos & 0xFF)[live] >= W).any() or ((pos >> 8)[live] >= H).any():
                raise ValueError("snapshot npc_pos: a live NPC outside the grid")

    def load_snapshot(self, snap: dict) -> None:
        """Writes host arrays (engine layout) into the device state (checked
        first: positions and layout indices the kernels would index with)."""
        self._check_snapshot(snap)
        if self.bank is not None and "p_layout" in snap:
            self.p_layout.copy_(torch.from_numpy(np.ascontiguousarray(snap["p_layout"], np.int16)))
        if self.sep_start is not None and "sep_start" in snap:
            self.sep_start.copy_(torch.from_numpy(np.ascontiguousarray(snap["sep_start"], np.int32)))
        if self.p_rpg is not None and "p_rpg" in snap:
            self.p_rpg.copy_(torch.from_numpy(np.ascontiguousarray(snap["p_rpg"], np.int32)))
        if self.item_pos is not None and "item_pos" in snap:
            self.item_pos.copy_(torch.from_numpy(
                np.ascontiguousarray(snap["item_pos"]).astype(np.uint16).view(np.int16)))
            self.item_mask.copy_(torch.from_numpy(
                np.ascontiguousarray(snap["item_mask"]).astype(np.uint32).view(np.int32)))
        if self.mt_py is not None:
            for f in ("mt_py", "mt_np", "dstore"):
                if f in snap:
                    a = np.ascontiguousarray(snap[f]).astype(np.uint32).view(np.int32)
                    getattr(self, f).copy_(torch.from_numpy(a.reshape(getattr(self, f).shape)))
        for f in STATE_FIELDS:
            if f not in snap:
                continue
            dst = getattr(self, f)
            a = np.ascontiguousarray(snap[f])
            if f == "npc_pos":
                a = a.astype(np.uint16).view(np.int16)
                if self.K == 0:
                    continue
                dst = dst[: self.K]
            elif f == "npc_health":
                if self.K == 0:
                    continue
                a = a.astype(np.int8)
                dst = dst[: self.K]
            elif f == "npc_alive":
                a = a.astype(np.uint32).view(np.int32)
            else:
                a = a.astype(np.int32)
            dst.copy_(torch.from_numpy(a.reshape(dst.shape)))
        if self.npc_grid is not None and ("npc_pos" in snap or "npc_alive" in snap):
            self._rebuild_npc_grid()

    def _rebuild_npc_grid(self) -> None:
        """Dense NPCs: the occupancy grid (slot + 1 per cell of the NPC depth)
        from npc_pos / npc_alive, after state was written from the host."""
        from .enums import npc_alive_bits
        K, B, H = self.K, self.B, int(self.cfg.height)
        pos = self.npc_pos[:K].cpu().numpy().view(np.uint16).astype(np.int64)
        live = npc_alive_bits(self.npc_alive.cpu().numpy().view(np.uint32), K)
        grid = np.zeros((B, int(self.cfg.width) * H), np.uint8)
        k, g = np.nonzero(live)
        grid[g, (pos[k, g] & 0xFF) * H + (pos[k, g] >> 8)] = (k + 1).astype(np.uint8)
        self.npc_grid.copy_(torch.from_numpy(grid))

    # -- checkpoint / resume -------------------------------------------------
    def save(self, path) -> None:
        """Checkpoint: the whole SoA state (snapshot()) with the configuration,
        seed and game offset, as one .npz (the reference's counterpart is a
        GameState.to_prims snapshot per game, state.py:94-132)."""
        import json
        snap = self.snapshot()
        extra = {} if self.cfg.layouts is None else {"layouts": np.asarray(self.cfg.layouts)}
        np.savez(path, cfg_json=np.frombuffer(json.dumps(self.cfg.to_dict()).encode(), np.uint8),
                 seed=np.array([self.seed], np.uint64),
                 game_offset=np.array([self.game_offset], np.int64), **extra, **snap)

    @classmethod
    def load(cls, path, device: Optional[torch.device] = None) -> "BatchedEngine":
        """Resume from save(): a new engine whose state, and therefore every
        later tick, equals the saved one's."""
        import json
        z = np.load(path, allow_pickle=False)
        cfg = EnvConfig.from_dict(json.loads(bytes(z["cfg_json"]).decode()),
                                  layouts=z["layouts"] if "layouts" in z.files else None)
        n = int(np.asarray(z["tick"]).shape[-1])
        eng = cls(cfg, n, seed=int(z["seed"][0]), game_offset=int(z["game_offset"][0]),
                  device=device, reset=False)
        eng.load_snapshot({k: z[k] for k in z.files})
        return eng

    def dungeon_stairs(self, games, episodes, depths, gens) -> np.ndarray:
        """Staircase and layout of (local game, episode, depth, generation)
        dungeons via orx_dungeon_spawn; returns int32 [n, 3] (sx, sy, layout;
        layout -1 for EmptyDungeonGenerator)."""
        n = len(games)
        if n == 0:
            return np.zeros((0, 3), np.int32)
        t = lambda a, dt: torch.as_tensor(np.asarray(a), dtype=dt).to(self.device).contiguous()
        g = t(np.asarray(games, np.int64) + self.game_offset, torch.int64).to(torch.int32)
        e, d, gn = t(episodes, torch.int32), t(depths, torch.int32), t(gens, torch.int32)
        sx = torch.empty(n, dtype=torch.int32, device=self.device)
        sy = torch.empty_like(sx)
        lay = torch.empty_like(sx)
        with torch.cuda.device(self.device):
            code = self.lib.orx_dungeon_spawn(ctypes.byref(self._ccfg), ctypes.byref(self._st),
                                              _ptr(g), _ptr(e), _ptr(d), _ptr(gn), _ptr(sx),
                                              _ptr(sy), _ptr(lay), n, self.seed, self._stream())
        _lib.check("orx_dungeon_spawn", code)
        return torch.stack([sx, sy, lay], 1).cpu().numpy()

    def game_states(self, indices=None, full_world: bool = True, snap: Optional[dict] = None):
        """Reference-schema views (compat.GameStateView) of the given games; with
        ``full_world`` every dungeon of World.dungeons is materialized (depths
        no player stands on are regenerated on the GPU)."""
        from .compat import game_state, world_depths
        snap = self.snapshot() if snap is None else snap
        idx = range(self.B) if indices is None else indices
        extra = {}
        if full_world and self.dstore is not None:
            # stock-seed mode: the remembered dungeons are the world; a depth
            # no player stands on is in the ring of a player who entered it
            ds = snap["dstore"]
            n = ds.shape[1]
            c = self.cfg
            starts = (int(c.p1_depth), int(c.p2_depth)) if int(c.start_mode) == 2 else (0, 0)
            for i in idx:
                d1, d2 = int(snap["p_depth"][0][i]), int(snap["p_depth"][1][i])
                for d in world_depths(self.cfg, d1, d2):
                    if d in (d1, d2):
                        continue
                    for p, (s0, dp) in enumerate(zip(starts, (d1, d2))):
                        k = (d - s0) % n
                        if s0 <= d <= dp and int(ds[p, k, 0, i]) == d:
                            v = int(ds[p, k, 1, i])
                            break
                    else:
                        raise RuntimeError(f"game {i}: depth {d} not in the dungeon store")
                    extra.setdefault(i, {})[d] = (v & 0xFF, (v >> 8) & 0xFF, (v >> 16) - 1)
        elif full_world:
            req = []
            for i in idx:
                d1, d2 = int(snap["p_depth"][0][i]), int(snap["p_depth"][1][i])
                for d in world_depths(self.cfg, d1, d2):
                    if d not in (d1, d2):
                        req.append((i, d))
            st = self.dungeon_stairs([r[0] for r in req],
                                     [int(snap["episode"][r[0]]) for r in req],
                                     [r[1] for r in req], [0] * len(req))
            for (i, d), (x, y, lay) in zip(req, st):
                extra.setdefault(i, {})[d] = (int(x), int(y), int(lay))
        return [game_state(snap, i, self.cfg, extra.get(i, {}) if full_world else None,
                           bank=self.bank)
                for i in idx]

    def episode_returns(self) -> torch.Tensor:
        """(ret_sum, ep_count) stacked as int32 [2, n_games] (device)."""
        return torch.stack([self.ret_sum, self.ep_count])


# The shard streams, created once per device and shared by every
# StreamShardedEngine of the process: a HIP stream is bound to one of the
# process's few hardware queues when it is created, and a fresh pair per engine
# sometimes landed two shards (or a shard and the caller's stream) on one
# queue, where they run one after the other -- a two-shard step measured
# 132 us instead of 84-90 on one engine out of sixteen
# (profiles/r04_v11/stream_pairs.jsonl).  Reusing the first streams keeps every
# engine on the queues the first one got; their work is ordered by fork() and
# join() as before.
_SHARD_STREAMS: dict = {}


def shard_streams(device: torch.device, n: int) -> list:
    """The process's first ``n`` shard streams on ``device`` (created on first use)."""
    device = cuda_device(device)
    have = _SHARD_STREAMS.setdefault(device, [])
    while len(have) < n:
        have.append(torch.cuda.Stream(device=device))
    return have[:n]


class StreamShardedEngine:
    """One GPU's batch as ``n_streams`` shards, each a BatchedEngine on its
    own HIP stream (contiguous global game ids, ``parallel.shard``).

    The fused rollout is HBM-write-bound inside its tick loop, so what a
    launch loses is its ramp (state loads) and its tail (waves that took more
    rare ticks finish last, with too few waves left to keep HBM busy).  Launches
    on different streams run concurrently, so one shard's ramp and tail overlap
    the other shards' steady state.  A game's trajectory depends on its
    global id only (the Philox key), so the shards compute exactly what one
    engine over the whole batch computes (tests/test_gpu_parity.py).  This is
    the multi-GPU sharding of parallel.py applied within one device.
    """

    def __init__(self, cfg: EnvConfig, n_games: int, seed: int = 0, game_offset: int = 0,
                 device: Optional[torch.device] = None, n_streams: int = 2):
        from .parallel import shard
        self.device = cuda_device(device)
        self.B = int(n_games)
        n_streams = max(1, min(int(n_streams), self.B))
        self.streams = shard_streams(self.device, n_streams)
        self.parts = []
        cur = torch.cuda.current_stream(self.device)
        for k, s in enumerate(self.streams):
            off, cnt = shard(self.B, k, n_streams)
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                self.parts.append(BatchedEngine(cfg, cnt, seed=seed, game_offset=game_offset + off,
                                                device=self.device))
                self.parts[-1].concurrency = n_streams
        for s in self.streams:
            cur.wait_stream(s)

    def trajectory_buffers(self, n_ticks: int, obs_format: int = OBS_INT32):
        """Per-shard obs int32 [n_ticks, obs_rows(obs_format), count] and act
        int8 [n_ticks, count, 2]."""
        return ([torch.empty((n_ticks, obs_rows(obs_format), e.B), dtype=torch.int32,
                             device=self.device) for e in self.parts],
                [torch.empty((n_ticks, e.B, 2), dtype=torch.int8, device=self.device)
                 for e in self.parts])

    def rollout_launcher(self, n_ticks: int, p1: int = Policy.Random, p2: int = Policy.Random,
                         obs=None, act=None, obs_format: int = OBS_INT32):
        """A zero-argument callable launching every shard's rollout on its own
        stream (``obs``/``act``: per-shard lists, or None).  Ordering against
        the caller's stream is explicit: ``fork()`` before (the shards wait for
        the caller's work so far), ``join()`` after (the caller waits for the
        shards) -- a fork per launch would put a cross-queue barrier between
        consecutive launches of a shard."""
        obs = obs or [None] * len(self.parts)
        act = act or [None] * len(self.parts)
        go = []
        for e, s, o, a in zip(self.parts, self.streams, obs, act):
            with torch.cuda.stream(s):
                go.append(e.rollout_launcher(n_ticks, p1, p2, obs=o, act=a,
                                             obs_format=obs_format))

        def launch():
            for g in go:
                g()
        return launch

    def split_log(self, log: torch.Tensor) -> list:
        """A move log int8 [T, n_games, 2] as per-shard contiguous logs (copies)."""
        from .parallel import shard
        out = []
        for k, e in enumerate(self.parts):
            off, cnt = shard(self.B, k, len(self.parts))
            out.append(log[:, off:off + cnt].contiguous())
        return out

    def replay_launcher(self, logs, obs=None, obs_format: int = OBS_INT32):
        """A zero-argument callable replaying every shard's move log (orx_step_n;
        ``logs``: per-shard int8 [T, count, 2] as ``split_log`` makes them,
        ``obs``: per-shard row buffers or None) on the shard's own stream;
        ordered against the caller's stream by ``fork()`` / ``join()`` as
        ``rollout_launcher``.  Results equal one engine's orx_step_n over the
        whole log (tests/test_gpu_parity.py)."""
        obs = obs or [None] * len(self.parts)
        if len(logs) != len(self.parts) or len(obs) != len(self.parts):
            raise ValueError(f"one log and one row buffer per shard ({len(self.parts)})")

        def launch():
            for e, s, l, o in zip(self.parts, self.streams, logs, obs):
                with torch.cuda.stream(s):
                    e.step_n(l, obs=o, obs_format=obs_format)
        return launch

    def fork(self) -> None:
        """Every shard's stream waits for the caller's current stream's work so far."""
        cur = torch.cuda.current_stream(self.device)
        for s in self.streams:
            s.wait_stream(cur)

    def join(self) -> None:
        """The caller's current stream waits for every shard's work so far."""
        cur = torch.cuda.current_stream(self.device)
        for s in self.streams:
            cur.wait_stream(s)

    def rollout_lanes(self) -> int:
        return self.parts[0].rollout_lanes()

    def rollout_shape(self, p1: int = Policy.Random, p2: int = Policy.Random,
                      trajectory: bool = True) -> dict:
        """The shape each shard's concurrent rollout launch takes (the first shard's)."""
        return self.parts[0].rollout_shape(p1, p2, trajectory)

    def episode_returns(self) -> torch.Tensor:
        """(ret_sum, ep_count) int32 [2, n_games] in global id order (device)."""
        self.join()
        return torch.cat([e.episode_returns() for e in self.parts], dim=1)

    def snapshot(self) -> dict:
        """The whole batch's SoA state, shards concatenated along the game axis."""
        self.join()
        snaps = [e.snapshot() for e in self.parts]
        return {k: np.concatenate([s[k] for s in snaps], axis=snaps[0][k].ndim - 1)
                for k in snaps[0]}
