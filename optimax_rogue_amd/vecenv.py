"""VecEnv: the learner-facing batched environment over BatchedEngine.

The reference runs one game per server process and hands each bot a
``GameState`` view every tick (server/main.py:110-113,
optimax_rogue_bots/main.py:118-155).  A learner over hundreds of thousands of
games wants tensors instead: this wraps the engine's C-ABI calls in the
usual reset / step / rollout shape, everything resident on the GPU.

* observation: int32 [n_games, 14], the fields of ``OBS_FIELDS`` (the same
  row ``orx_rollout`` writes per tick);
* reward: float32 [n_games], player 1's view: +1 Player1Win, -1 Player2Win,
  0 otherwise, on the step that ends an episode;
* done: bool [n_games], that step.  The step after ``done`` starts the game's
  next episode (the engine's autoreset: that step's actions are not played).

Player 2 is the learner's opponent: a device policy (``Policy.Random``,
``Policy.Staircase``, ``Policy.Stay``), or ``None`` for self-play, where
``step`` takes both players' actions.
"""
from __future__ import annotations

import warnings
from typing import Optional, Union

import torch

from .config import EnvConfig
from .engine import BatchedEngine
from .enums import EXT_HEAL, OBS_FIELDS, STATUS_BAD_ACTION, Policy, UpdateResult

_STATUS = OBS_FIELDS.index("status")


class VecEnv:
    """reset / step / rollout over one BatchedEngine.

    ``check_actions`` -- what happens to actions outside the Move codes (e.g.
    a 0-based argmax); the engine always stops such a game with
    STATUS_BAD_ACTION (done, reward 0: a truncation; it restarts on the next
    step), and the step returns normally:

    * ``"deferred"`` (default): the launch also counts refused actions into a
      device counter, and every ``check_every`` steps ``step`` reads it back
      asynchronously (pinned memory and an event, no host sync); once a read
      that has landed shows new refusals, ``step`` issues a RuntimeWarning
      (and ``warnings_seen`` counts it).  Nothing is raised and every tick is
      played.  When a read has not landed at its check, the next check waits
      for it, so the warning comes some check periods after the refusal --
      how many depends on when the copy completes.  ``bad_actions()`` reads
      the exact count now (synchronizing).
    * ``"deferred-raise"``: as ``"deferred"``, but the ``step`` that sees new
      refusals raises ValueError instead of warning -- before launching, so
      the actions passed to THAT call are not played (pass them again after
      handling the error).
    * ``True``: a host check before every launch raises ValueError at once
      (a device-to-host sync per step; the offending call plays no tick).
    * ``False``: no detection.

    ``out_buffers`` -- 0 (default): every step returns fresh tensors; k > 0:
    the outputs come from a ring of k preallocated sets, so a step's tensors
    are overwritten k steps later (copy what must outlive that); this spares
    four allocations per step on the eager path.
    """

    def __init__(self, cfg: EnvConfig, n_games: int, seed: int = 0, game_offset: int = 0,
                 device: Optional[torch.device] = None,
                 opponent: Optional[int] = Policy.Random,
                 check_actions: Union[bool, str] = "deferred", out_buffers: int = 0,
                 check_every: int = 64):
        if not int(cfg.autoreset):
            raise ValueError("VecEnv needs cfg.autoreset = 1 (finished games restart)")
        if isinstance(check_actions, str):
            if check_actions not in ("deferred", "deferred-raise"):
                raise ValueError('check_actions must be a bool, "deferred" or "deferred-raise"')
        elif type(check_actions).__name__ in ("bool", "bool_") or check_actions in (0, 1):
            check_actions = bool(check_actions)   # (1, np.True_ -> True: the host check)
        else:
            raise ValueError('check_actions must be a bool, "deferred" or "deferred-raise"')
        self.engine = BatchedEngine(cfg, n_games, seed=seed, game_offset=game_offset,
                                    device=device)
        self.B = self.engine.B
        self.device = self.engine.device
        self.opponent = None if opponent is None else int(opponent)
        self.check_actions = check_actions
        self.check_every = max(1, int(check_every))
        self.out_buffers = max(0, int(out_buffers))
        self._init_step_consts()

    def _init_step_consts(self) -> None:
        """Per-call constants of step() (its Python cost is the eager path's)."""
        self._shape1 = torch.Size([self.B])
        self._shape2 = torch.Size([self.B, 2])
        self._obs_shape = (self.B, len(OBS_FIELDS))
        self._p2 = int(Policy.NONE if self.opponent is None else self.opponent)
        # refused-action counter (device) and its asynchronous read-back
        self._bad_dev = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._bad_ptr = self._bad_dev.data_ptr()
        self._bad_host = torch.zeros(1, dtype=torch.int32).pin_memory() \
            if isinstance(self.check_actions, str) else None
        self._bad_event = None
        self._bad_seen = 0
        self.warnings_seen = 0
        self._steps = 0
        self._ring = [self._alloc_out() for _ in range(self.out_buffers)]
        self._ring_launch = [None] * len(self._ring)   # their prebuilt launches (first use)
        self._slot = 0
        self._stock = None   # stock-seed mode (orx_policy + orx_step per tick)
        self._fresh_launch = None   # the argument-block launch for fresh outputs

    def _alloc_out(self):
        d = self.device
        return (torch.empty(self._obs_shape, dtype=torch.int32, device=d),
                torch.empty(self.B, dtype=torch.float32, device=d),
                torch.empty(self.B, dtype=torch.bool, device=d),
                torch.empty(self.B, dtype=torch.int32, device=d))

    # -- observation -----------------------------------------------------------
    def observe(self) -> torch.Tensor:
        """The current observation rows, int32 [n_games, 14] (OBS_FIELDS order)."""
        e = self.engine
        return torch.stack([e.p_x[0], e.p_y[0], e.p_depth[0], e.p_health[0],
                            e.p_x[1], e.p_y[1], e.p_depth[1], e.p_health[1],
                            e.tick, e.status, e.st_x[0], e.st_y[0], e.st_x[1], e.st_y[1]], dim=1)

    @staticmethod
    def outcome(before: torch.Tensor, after: torch.Tensor):
        """(reward, done) of a transition between two status tensors.  A game
        that leaves InProgress for an engine stop code (>= 16: a bad action, an
        exhausted random stream) is done too, with reward 0 -- a truncation:
        the engine's autoreset starts its next episode on the following step,
        so the learner must see this one end."""
        done = (before == UpdateResult.InProgress) & (after >= UpdateResult.Player1Win) \
            & ((after <= UpdateResult.Tie) | (after >= STATUS_BAD_ACTION))
        reward = torch.where(done, (after == UpdateResult.Player1Win).float()
                             - (after == UpdateResult.Player2Win).float(),
                             torch.zeros((), device=after.device))
        return reward, done

    # -- refused actions ---------------------------------------------------------
    def bad_actions(self) -> int:
        """Games whose actions were refused (outside the Move codes) since this
        VecEnv was made, by orx_env_step (synchronizes)."""
        return int(self._bad_dev.item())

    def _bad_message(self, n: int) -> str:
        return (f"{n} game(s) got actions outside the Move values 1..{self._max_move()} (an "
                "argmax over logits is 0-based: add 1); the engine stopped them with "
                "STATUS_BAD_ACTION (done, reward 0)")

    def _poll_bad(self) -> None:
        """Deferred check: reads the counter's last asynchronous copy if it
        has landed, raises on new refusals, and queues the next copy."""
        if torch.cuda.is_current_stream_capturing():
            return
        ev = self._bad_event
        if ev is not None:
            if not ev.query():
                return
            n = int(self._bad_host[0])
            self._bad_event = None
            if n > self._bad_seen:
                new, self._bad_seen = n - self._bad_seen, n
                if self.check_actions == "deferred-raise":
                    raise ValueError(self._bad_message(new))
                self.warnings_seen += 1
                warnings.warn(self._bad_message(new), RuntimeWarning, stacklevel=3)
        # the copy runs on the counter's device's current stream (the stream
        # orx_env_step_ex launches on), and the event is recorded there, not
        # on whichever device happens to be current
        self._bad_host.copy_(self._bad_dev, non_blocking=True)
        self._bad_event = torch.cuda.Event()
        self._bad_event.record(torch.cuda.current_stream(self.device))

    # -- reset / step / rollout ----------------------------------------------------
    def reset(self, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Starts the masked games (all if None) at their NEXT episode's setup:
        each game's episode index advances by one, so a truncated game gets a
        fresh dungeon and fresh draws (randomness is keyed on game, episode
        and tick), and two resets in a row give different starts.  A truncated
        episode has no outcome: it does not count in the engine's episode
        returns (ret_sum / ep_count)."""
        e = self.engine
        if mask is not None:
            mask = mask.to(self.device).bool().reshape(-1)
            if mask.numel() != self.B:
                raise ValueError("mask must have n_games elements")
        e.reset(mask, episode=e.episode + 1)
        return self.observe()

    def _max_move(self) -> int:
        return 6 if int(self.engine.cfg.flags) & EXT_HEAL else 5

    def step(self, actions: torch.Tensor):
        """Plays one tick: ``actions`` integer [n_games] (player 1; the opponent
        policy moves player 2) or [n_games, 2] (self-play), Move values 1..5
        (1..6 with EXT_HEAL), any integer dtype.  A value outside them (e.g. a
        0-based argmax) stops that game with STATUS_BAD_ACTION: it is done
        with reward 0 this step (a truncation) and restarts on the next one;
        ``check_actions`` decides whether and when it is reported (a
        warning by default; class docstring).  One launch (orx_env_step_ex) and no host sync
        (unless check_actions=True).  Returns (observation int32 [n_games,
        14], reward float32, done bool, status int32 [n_games]): separate
        tensors, fresh ones unless ``out_buffers`` > 0."""
        shape = actions.shape
        if shape != self._shape1 and shape != self._shape2:   # no silent broadcasting
            raise ValueError(f"actions must be [n_games] or [n_games, 2], got {tuple(shape)}")
        nb = BatchedEngine._ACTION_BYTES.get(actions.dtype)
        if nb is None:
            raise ValueError(f"actions must be an integer tensor, got {actions.dtype}")
        if self.opponent is None and len(shape) == 1:
            raise ValueError("self-play (opponent=None) takes [n_games, 2] actions")
        a = actions if actions.device == self.device else actions.to(self.device)
        if not a.is_contiguous():
            a = a.contiguous()
        if self.check_actions is True:
            hi = self._max_move()
            if bool(((a < 1) | (a > hi)).any()):
                raise ValueError(f"actions must be Move values 1..{hi} (an argmax over logits is "
                                 "0-based: add 1)")
        if self._stock is None:   # (decided at the first step)
            self._stock = getattr(self.engine, "mt_py", None) is not None
        if self._stock:   # stock-seed mode
            return self._step_stock(a)
        deferred = self._bad_host is not None
        bad = self._bad_ptr if deferred else None
        if deferred:   # (before the launch: a call that raises plays no tick)
            self._steps += 1
            if self._steps % self.check_every == 0:
                self._poll_bad()
        if self._ring:
            k = self._slot
            out = self._ring[k]
            self._slot = (k + 1) % len(self._ring)
            go = self._ring_launch[k]
            if go is None:   # one prebuilt argument block per output set
                go = self._ring_launch[k] = self.engine.env_step_slot(
                    self._p2, *out, self._bad_dev if deferred else None)
            go(a.data_ptr(), nb, len(shape))
        else:
            out = self._alloc_out()
            obs, reward, done, status = out
            if self._fresh_launch is None:   # one argument block, its outputs set per call
                self._fresh_launch = self.engine.env_step_slot(
                    self._p2, *out, self._bad_dev if deferred else None)
            self._fresh_launch(a.data_ptr(), nb, len(shape),
                               (obs.data_ptr(), reward.data_ptr(), done.data_ptr(),
                                status.data_ptr()))
        return out

    def _step_stock(self, a: torch.Tensor):
        """Stock-seed mode (the bots draw from each game's own MT19937 stream):
        orx_policy + orx_step, invalid values mapped on the device to the
        invalid move 0 before the int8 cast (257 must not wrap to 1)."""
        e = self.engine
        hi = self._max_move()
        a = torch.where((a >= 1) & (a <= hi), a, torch.zeros((), dtype=a.dtype,
                                                             device=a.device)).to(torch.int8)
        if a.dim() == 1:
            e.actions[:, 0].copy_(a)
            e.policy(Policy.NONE, self.opponent)   # player 2's move; player 1's kept
        else:
            e.actions.copy_(a)
        before = e.status.clone()
        status = e.step(e.actions).clone()
        reward, done = self.outcome(before, status)
        if self._bad_host is not None:   # the deferred check, counted with torch ops here
            self._bad_dev += ((before == UpdateResult.InProgress)
                              & (status == STATUS_BAD_ACTION)).sum(dtype=torch.int32)
            self._steps += 1
            if self._steps % self.check_every == 0:
                self._poll_bad()
        return self.observe(), reward, done, status

    def rollout(self, n_ticks: int, p1: int = Policy.Random, p2: Optional[int] = None) -> dict:
        """``n_ticks`` ticks with device policies for both players in one fused
        launch (orx_rollout).  Returns obs int32 [T, 14, n_games], act int8
        [T, n_games, 2], reward float32 [T, n_games], done bool [T, n_games]."""
        p2 = self.opponent if p2 is None else int(p2)
        if p2 is None:
            raise ValueError("rollout needs a policy for player 2")
        e = self.engine
        obs = torch.empty((n_ticks, len(OBS_FIELDS), self.B), dtype=torch.int32, device=self.device)
        act = torch.empty((n_ticks, self.B, 2), dtype=torch.int8, device=self.device)
        before = e.status.clone()
        e.rollout(n_ticks, int(p1), p2, obs=obs, act=act)
        status = obs[:, _STATUS]
        prev = torch.cat([before[None], status[:-1]], dim=0)
        reward, done = self.outcome(prev, status)
        return {"obs": obs, "act": act, "reward": reward, "done": done}
