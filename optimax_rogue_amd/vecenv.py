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

from typing import Optional

import torch

from .config import EnvConfig
from .engine import BatchedEngine
from .enums import EXT_HEAL, OBS_FIELDS, STATUS_BAD_ACTION, Policy, UpdateResult

_STATUS = OBS_FIELDS.index("status")


class VecEnv:
    def __init__(self, cfg: EnvConfig, n_games: int, seed: int = 0, game_offset: int = 0,
                 device: Optional[torch.device] = None,
                 opponent: Optional[int] = Policy.Random, check_actions: bool = False):
        if not int(cfg.autoreset):
            raise ValueError("VecEnv needs cfg.autoreset = 1 (finished games restart)")
        self.engine = BatchedEngine(cfg, n_games, seed=seed, game_offset=game_offset,
                                    device=device)
        self.B = self.engine.B
        self.device = self.engine.device
        self.opponent = None if opponent is None else int(opponent)
        # True: step() raises ValueError on a non-Move action (a host check, so
        # every step synchronizes); False (default): the engine stops that game
        # with STATUS_BAD_ACTION, which step() reports as done (a truncation)
        self.check_actions = bool(check_actions)
        self._init_step_consts()

    def _init_step_consts(self) -> None:
        """Per-call constants of step() (its Python cost is the eager path's)."""
        self._shape1 = torch.Size([self.B])
        self._shape2 = torch.Size([self.B, 2])
        self._obs_shape = (self.B, len(OBS_FIELDS))
        self._p2 = int(Policy.NONE if self.opponent is None else self.opponent)

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
        with ``check_actions=True`` it raises ValueError instead (a host check:
        that step synchronizes).  One launch (orx_env_step) and no host sync
        otherwise.  Returns (observation, reward, done, status), all fresh
        tensors (status is the observation's status column, a view)."""
        e = self.engine
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
        if self.check_actions:
            hi = self._max_move()
            if bool(((a < 1) | (a > hi)).any()):
                raise ValueError(f"actions must be Move values 1..{hi} (an argmax over logits is "
                                 "0-based: add 1)")
        if e.mt_py is not None:
            return self._step_stock(a)
        obs = torch.empty(self._obs_shape, dtype=torch.int32, device=self.device)
        reward = torch.empty(self.B, dtype=torch.float32, device=self.device)
        done = torch.empty(self.B, dtype=torch.bool, device=self.device)
        e._env_step_raw(a, nb, self._p2, obs, reward, done)
        return obs, reward, done, obs[:, _STATUS]

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
