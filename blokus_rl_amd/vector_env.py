"""Config 5: the PPO Blokus vector env on the GPU (bk_vec_reset / bk_vec_step).

A gymnasium-style vector env replacing `gym.vector.SyncVectorEnv([blokus-simple-v0] * E)` in the
reference PPO trainer (ppo/trainer.py:36-38, `_play_env` :128-175): 7x7, the agent (colour 0)
against a built-in uniform-random opponent (colour 1), reward +1 / 0 / -1 at the end, auto-reset.
Every step is one fused kernel launch for all E envs. The legal-move mask the reference builds
in a Python loop from `envs.get_attr("ai_possible_indexes")` and `FilterLegalMoves`
(ppo/trainer.py:380-386, ppo/agent.py:33-42) comes back as a device tensor, `valid_mask()`.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from .engine import Engine, _check, _ptr


class BlokusVectorEnv:
    def __init__(self, num_envs: int, board_size: int = 7, max_piece_cells: int = 4,
                 device: str | torch.device | None = None):
        self.eng = Engine(board_size, 2, max_piece_cells, device=device)
        self.num_envs = E = num_envs
        dev = self.eng.device
        self.device = dev
        self.single_action_space_n = self.eng.A
        self.states = torch.empty((E, 384), dtype=torch.uint8, device=dev)
        self.rng = torch.zeros(E, dtype=torch.int64, device=dev)
        self.obs = torch.empty((E, board_size, board_size), dtype=torch.uint8, device=dev)
        self.mask_words = torch.empty((E, self.eng.W), dtype=torch.int64, device=dev)
        self.reward = torch.zeros(E, dtype=torch.float32, device=dev)
        self.done = torch.zeros(E, dtype=torch.int32, device=dev)
        self.actions = torch.zeros(E, dtype=torch.int32, device=dev)  # bk_vec_policy's draws
        self.logp = torch.zeros(E, dtype=torch.float32, device=dev)

    def _s(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def reset(self, seed: int | None = None):
        seeds = torch.from_numpy(
            np.array([(0 if seed is None else seed) * 1_000_003 + e for e in range(self.num_envs)], dtype=np.int64)
        ).to(self.device)
        _check(self.eng.lib.bk_vec_reset(self.eng.h, _ptr(self.states), _ptr(self.rng), _ptr(seeds), self.num_envs,
                                         _ptr(self.obs), _ptr(self.mask_words), self._s()))
        return self.obs, {}

    def step(self, actions: torch.Tensor | None):
        """actions [E] int32 on the device (None: random legal agent moves drawn in-kernel)."""
        act = None if actions is None else actions.to(device=self.device, dtype=torch.int32).contiguous()
        _check(self.eng.lib.bk_vec_step(self.eng.h, _ptr(self.states), _ptr(self.rng), _ptr(act), self.num_envs,
                                        _ptr(self.obs), _ptr(self.mask_words), _ptr(self.reward), _ptr(self.done),
                                        self._s()))
        term = self.done.bool()
        return self.obs, self.reward, term, torch.zeros_like(term), {}

    def step_raw(self, actions: torch.Tensor | None = None):
        """The env step alone (one bk_vec_step launch, no result tensors built): obs, mask_words,
        reward and done are updated in place. Capturable in a HIP graph (the checks are host-side)."""
        act = actions
        if act is not None:
            if not (act.is_cuda and act.device == torch.device(self.device) and act.dtype == torch.int32
                    and act.is_contiguous() and act.numel() == self.num_envs):
                raise ValueError("step_raw wants a contiguous int32 [num_envs] tensor on the env's device")
        _check(self.eng.lib.bk_vec_step(self.eng.h, _ptr(self.states), _ptr(self.rng), _ptr(act), self.num_envs,
                                        _ptr(self.obs), _ptr(self.mask_words), _ptr(self.reward), _ptr(self.done),
                                        self._s()))

    def sample_policy(self, logits: torch.Tensor, zero_masked: bool = True):
        """The agent's moves drawn from its policy on the device (bk_vec_policy): the rollout's
        `get_action_and_value(obs, possible_moves=...)` sample + log_prob (ppo/agent.py:148-156)
        over FilterLegalMoves (:27-42; zero_masked = its rule that a legal logit of exactly 0 is
        masked too) in one launch, from the actor's raw logits [E, A] f32 and the env's current
        legal-move bitmask. Returns (actions [E] int32, logp [E] f32), updated in place
        (capturable in a HIP graph: the checks are host-side)."""
        E, A = self.num_envs, self.eng.A
        if not (logits.is_cuda and logits.device == torch.device(self.device) and logits.dtype == torch.float32
                and logits.is_contiguous() and tuple(logits.shape) == (E, A)):
            raise ValueError(f"sample_policy wants contiguous float32 logits [{E}, {A}] on the env's device")
        _check(self.eng.lib.bk_vec_policy(self.eng.h, _ptr(logits), _ptr(self.mask_words), _ptr(self.rng), E,
                                          int(bool(zero_masked)), _ptr(self.actions), _ptr(self.logp), self._s()))
        return self.actions, self.logp

    def step_policy(self, logits: torch.Tensor, zero_masked: bool = True, fused: bool = True):
        """One rollout step on the device: the policy draw and the env step in ONE launch
        (bk_vec_step_policy: the draw reads the agent's legal mask from the step's own legality
        pass); fused=False: sample_policy then step_raw (two launches, the same results bit for
        bit). Returns (actions, logp) of the step; obs / mask_words / reward / done in place.
        Capturable in a HIP graph."""
        if not fused:
            self.sample_policy(logits, zero_masked)
            self.step_raw(self.actions)
            return self.actions, self.logp
        E, A = self.num_envs, self.eng.A
        if not (logits.is_cuda and logits.device == torch.device(self.device) and logits.dtype == torch.float32
                and logits.is_contiguous() and tuple(logits.shape) == (E, A)):
            raise ValueError(f"step_policy wants contiguous float32 logits [{E}, {A}] on the env's device")
        _check(self.eng.lib.bk_vec_step_policy(self.eng.h, _ptr(self.states), _ptr(self.rng), _ptr(logits),
                                               int(bool(zero_masked)), E, _ptr(self.obs), _ptr(self.mask_words),
                                               _ptr(self.reward), _ptr(self.done), _ptr(self.actions), _ptr(self.logp),
                                               self._s()))
        return self.actions, self.logp

    def valid_mask(self) -> torch.Tensor:
        """[E, A] bool: the agent's legal ids (the reference's ai_possible_indexes as a mask)."""
        return self.eng.unpack_mask(self.mask_words)

    def get_attr(self, name: str):
        if name == "ai_possible_indexes":
            m = self.valid_mask().cpu().numpy()
            return [np.nonzero(row)[0].tolist() for row in m]
        raise AttributeError(name)

    def masked_logits(self, logits: torch.Tensor) -> torch.Tensor:
        """FilterLegalMoves (ppo/agent.py:27-42) without the per-env Python loop: illegal ids at
        -1e9. (The reference also masks a legal logit that is exactly 0; this does not.)"""
        return torch.where(self.valid_mask(), logits, torch.full_like(logits, -1e9))
