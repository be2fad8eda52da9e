"""PPO trainer (blokus_rl/ppo/trainer.py:20-400) on the device vector env (config 5).

Rollouts never leave the GPU: BlokusVectorEnv steps all envs in one kernel and hands back the
agent's legal-move bitmask; the rollout's draw (FilterLegalMoves + Categorical sample + log_prob of
get_action_and_value, ppo/agent.py:27-42, 148-156) is one kernel over the actor's raw logits and
that bitmask (bk_vec_policy; `device_sampling=False` keeps the torch Categorical path); GAE is one kernel over
the [T, E] rollout (bk_ppo_gae, the reference's float32 operation order). The update
(`optimize_agent`) is the reference's clipped-surrogate PPO step — same minibatch order (it
draws its shuffles from np.random exactly as the reference does, so a seeded run matches),
advantage normalisation, clipped value loss, entropy bonus, grad-norm clipping, target-KL stop.
Hyper-parameter names are PPOHparams' (hparams.py:97-185).
"""
from __future__ import annotations

import ctypes
import time
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np
import torch
from torch import nn

from ..engine import _check, _ptr, _stream, load_library
from ..vector_env import BlokusVectorEnv
from .agent import get_agent


@dataclass
class PPOHparams:
    num_envs: int = 4
    agent_type: str = "mlp"
    save_interval: int = 100
    dropout: float = 0.1
    d_model: int = 64
    cnn_layers: int = 4
    cnn_channels: int = 1
    cnn_kernel_size: int = 3
    cnn_stride: int = 1
    cnn_padding: int = 1
    cnn_dropout: float = 0.1
    update_epochs: int = 4
    learning_rate: float = 2.5e-4
    total_timesteps: int = 500_000
    num_steps: int = 128
    num_minibatches: int = 4
    eps: float = 1e-5
    anneal_lr: bool = True
    gae: bool = True
    gamma: float = 0.99
    gae_lambda: float = 0.95
    clip_coef: float = 0.2
    norm_adv: bool = True
    clip_vloss: bool = True
    ent_coef: float = 0.01
    vf_coef: float = 0.5
    max_grad_norm: float = 0.5
    target_kl: float | None = 0.01
    # env preset (blokus-simple-v0: 7x7, 2 players, pieces of <= 4 cells -> 919 ids)
    board_size: int = 7
    max_piece_cells: int = 4
    seed: int = 42
    cuda: bool = True
    checkpoint_dir: Path = Path("models/checkpoints")
    extra: dict = field(default_factory=dict)

    def __post_init__(self):
        self.checkpoint_dir = Path(self.checkpoint_dir)
        self.batch_size = self.num_envs * self.num_steps
        self.minibatch_size = self.batch_size // self.num_minibatches
        self.num_updates = self.total_timesteps // self.batch_size

    @classmethod
    def from_dict(cls, d: dict) -> "PPOHparams":
        known = set(cls.__dataclass_fields__)
        hp = cls(**{k: v for k, v in d.items() if k in known})
        hp.extra = {k: v for k, v in d.items() if k not in known}
        return hp


def compute_gae(rewards, values, dones, next_value, next_done, gamma: float, gae_lambda: float):
    """_compute_gae (trainer.py:177-211) + returns (:83) on the device: -> (advantages, returns)."""
    T, E = rewards.shape
    dev = rewards.device
    f = lambda t: t.to(device=dev, dtype=torch.float32).contiguous()  # noqa: E731
    rewards, values, dones = f(rewards), f(values), f(dones)
    nv, nd = f(next_value).view(-1), f(next_done).view(-1)
    adv = torch.empty_like(rewards)
    ret = torch.empty_like(rewards)
    _check(load_library().bk_ppo_gae(T, E, _ptr(rewards), _ptr(values), _ptr(dones), _ptr(nv), _ptr(nd),
                                     ctypes.c_float(gamma), ctypes.c_float(gamma * gae_lambda), _ptr(adv), _ptr(ret),
                                     _stream(dev)))
    return adv, ret


class Memory:
    """ppo/memory.py:7-62 on the device."""

    def __init__(self, T: int, E: int, obs_shape, device):
        z = lambda *s: torch.zeros((T, E) + tuple(s), device=device)  # noqa: E731
        self.obs_shape = tuple(obs_shape)
        self.obs = z(*obs_shape)
        self.actions = z()
        self.logprobs, self.rewards, self.dones, self.values = z(), z(), z(), z()
        self.advantages, self.returns = z(), z()

    def get_flatten_batch(self):
        return {"obs": self.obs.reshape((-1,) + self.obs_shape), "logprobs": self.logprobs.reshape(-1),
                "actions": self.actions.reshape(-1), "advantages": self.advantages.reshape(-1),
                "returns": self.returns.reshape(-1), "values": self.values.reshape(-1)}


def optimize_agent(agent: nn.Module, optimizer, batch: dict, hp) -> dict:
    """_optimize_agent (trainer.py:213-311): update_epochs passes of shuffled minibatches of the
    clipped PPO objective; returns the reference's logged values of the last minibatch."""
    b_inds = np.arange(hp.batch_size)
    clipfracs = []
    for _ in range(hp.update_epochs):
        np.random.shuffle(b_inds)
        for start in range(0, hp.batch_size, hp.minibatch_size):
            mb = torch.as_tensor(b_inds[start:start + hp.minibatch_size], dtype=torch.long,
                                 device=batch["obs"].device)
            _, newlogprob, entropy, newvalue = agent.get_action_and_value(batch["obs"][mb],
                                                                          batch["actions"].long()[mb])
            logratio = newlogprob - batch["logprobs"][mb]
            ratio = logratio.exp()
            with torch.no_grad():
                old_approx_kl = (-logratio).mean()
                approx_kl = ((ratio - 1) - logratio).mean()
                clipfracs.append(((ratio - 1.0).abs() > hp.clip_coef).float().mean().item())
            adv = batch["advantages"][mb]
            if hp.norm_adv:
                adv = (adv - adv.mean()) / (adv.std() + 1e-8)
            pg_loss = torch.max(-adv * ratio, -adv * torch.clamp(ratio, 1 - hp.clip_coef, 1 + hp.clip_coef)).mean()
            newvalue = newvalue.view(-1)
            ret, val = batch["returns"][mb], batch["values"][mb]
            if hp.clip_vloss:
                unclipped = (newvalue - ret) ** 2
                clipped = (val + torch.clamp(newvalue - val, -hp.clip_coef, hp.clip_coef) - ret) ** 2
                v_loss = 0.5 * torch.max(unclipped, clipped).mean()
            else:
                v_loss = 0.5 * ((newvalue - ret) ** 2).mean()
            entropy_loss = entropy.mean()
            loss = pg_loss - hp.ent_coef * entropy_loss + v_loss * hp.vf_coef
            optimizer.zero_grad()
            loss.backward()
            nn.utils.clip_grad_norm_(agent.parameters(), hp.max_grad_norm)
            optimizer.step()
        if hp.target_kl is not None and approx_kl > hp.target_kl:
            break
    y_pred, y_true = batch["values"].cpu().numpy(), batch["returns"].cpu().numpy()
    var_y = np.var(y_true)
    explained_var = np.nan if var_y == 0 else 1 - np.var(y_true - y_pred) / var_y
    return {"learning_rate": optimizer.param_groups[0]["lr"], "loss": loss.item(), "value_loss": v_loss.item(),
            "policy_loss": pg_loss.item(), "entropy": entropy_loss.item(), "old_approx_kl": old_approx_kl.item(),
            "approx_kl": approx_kl.item(), "clipfrac": float(np.mean(clipfracs)), "explained_variance": explained_var}


class PPOTrainer:
    """PPOTrainer (trainer.py:20-400) with the device vector env instead of SyncVectorEnv."""

    def __init__(self, hparams: PPOHparams, device: str | torch.device | None = None, device_sampling: bool = True,
                 channels_last: bool = False, phase_timers: bool = False):
        """device_sampling: the rollout's draw in one kernel (bk_vec_policy) instead of torch's
        Categorical; channels_last: the cnn agent's convolutions in NHWC (off by default: measured
        round 6, MIOPEN_FIND_MODE=FAST, 8192 envs, 23.1 s per update against 2.0 s in NCHW — MIOpen
        then picks composable-kernel grouped convolutions instead of its NCHW implicit GEMMs;
        parameters and checkpoint keys are the same either way); phase_timers: synchronize and accumulate rollout / update seconds in
        self.phase_s (benchmarking)."""
        self.hparams = hp = hparams
        self.device_sampling = device_sampling
        self.phase_timers = phase_timers
        self.phase_s = {"rollout": 0.0, "gae": 0.0, "update": 0.0}
        self.envs = BlokusVectorEnv(hp.num_envs, hp.board_size, hp.max_piece_cells, device=device)
        self.device = self.envs.device
        self.obs_shape = (hp.board_size, hp.board_size)
        self.agent = get_agent(hp.agent_type)(self.obs_shape, self.envs.single_action_space_n, hp).to(self.device)
        if channels_last and hp.agent_type == "cnn":
            self.agent = self.agent.to(memory_format=torch.channels_last)
        self.optimizer = torch.optim.Adam(self.agent.parameters(), lr=hp.learning_rate, eps=hp.eps)
        self.memory = Memory(hp.num_steps, hp.num_envs, self.obs_shape, self.device)
        self.global_step = 0
        self.update = 1
        self.total_episodes = 0
        self.total_episodes_reward = 0.0
        self.logs: list[dict] = []
        self._ep_ret = torch.zeros(hp.num_envs, device=self.device)
        self._ep_count = torch.zeros((), device=self.device)
        self._ep_sum = torch.zeros((), device=self.device)

    def _compute_anneal_lr(self, update: int) -> float:
        """trainer.py:113-126."""
        return (1.0 - (update - 1.0) / self.hparams.num_updates) * self.hparams.learning_rate

    def _play_env(self, next_obs, next_done):
        """trainer.py:128-175: num_steps vector steps, all on the device."""
        hp, m = self.hparams, self.memory
        for step in range(hp.num_steps):
            self.global_step += hp.num_envs
            m.obs[step] = next_obs
            m.dones[step] = next_done
            with torch.inference_mode():
                if self.device_sampling:
                    h = self.agent.features(next_obs)
                    logits = self.agent.actor(h).float().contiguous()  # raw: the filter runs in the draw
                    value = self.agent.critic(h)
                else:
                    action, logproba, _, value = self.agent.get_action_and_value(
                        next_obs, possible_moves=self.envs.mask_words)
                m.values[step] = value.flatten()
            if self.device_sampling:  # the draw and the env step in one launch (bk_vec_step_policy)
                action, logproba = self.envs.step_policy(logits, zero_masked=True)
                obs, reward, term = self.envs.obs, self.envs.reward, self.envs.done.bool()
            else:
                obs, reward, term = None, None, None
            m.actions[step] = action
            m.logprobs[step] = logproba
            if not self.device_sampling:
                obs, reward, term, _, _ = self.envs.step(action)
            m.rewards[step] = reward.view(-1)
            next_obs, next_done = obs.float(), term.float()
            self._ep_ret += reward
            self._ep_count += next_done.sum()
            self._ep_sum += (self._ep_ret * next_done).sum()
            self._ep_ret *= 1.0 - next_done
        return next_obs, next_done

    def _compute_gae(self, next_value, next_done):
        m = self.memory
        adv, ret = compute_gae(m.rewards, m.values, m.dones, next_value, next_done, self.hparams.gamma,
                               self.hparams.gae_lambda)
        return adv, ret

    def train(self, num_updates: int | None = None):
        hp = self.hparams
        t0 = time.time()
        obs, _ = self.envs.reset(seed=hp.seed)
        next_obs = obs.float()
        next_done = torch.zeros(hp.num_envs, device=self.device)
        last = self.update + (num_updates or hp.num_updates)
        for update in range(self.update, last):
            if hp.anneal_lr:
                self.optimizer.param_groups[0]["lr"] = self._compute_anneal_lr(update)
            t0p = self._tick()
            next_obs, next_done = self._play_env(next_obs, next_done)
            with torch.inference_mode():
                next_value = self.agent.get_value(next_obs).reshape(1, -1)
            t1p = self._tick("rollout", t0p)
            self.memory.advantages, self.memory.returns = self._compute_gae(next_value, next_done)
            t2p = self._tick("gae", t1p)
            log = optimize_agent(self.agent, self.optimizer, self.memory.get_flatten_batch(), hp)
            self._tick("update", t2p)
            log["SPS"] = int(self.global_step / max(time.time() - t0, 1e-9))
            self.logs.append(log)
            if update % hp.save_interval == 0:
                self._save_checkpoint(update)
            self.update += 1
        self.total_episodes = int(self._ep_count.item())
        self.total_episodes_reward = float(self._ep_sum.item())
        return self.logs

    def _tick(self, phase: str | None = None, since: float = 0.0) -> float:
        if not self.phase_timers:
            return 0.0
        torch.cuda.synchronize(self.device)
        now = time.perf_counter()
        if phase is not None:
            self.phase_s[phase] += now - since
        return now

    @property
    def mean_episode_reward(self) -> float:
        return self.total_episodes_reward / self.total_episodes if self.total_episodes else 0.0

    def _save_checkpoint(self, update: int):
        """trainer.py:352-363 (same keys)."""
        self.hparams.checkpoint_dir.mkdir(parents=True, exist_ok=True)
        torch.save({"agent": self.agent.state_dict(), "optimizer": self.optimizer.state_dict(), "update": update,
                    "global_step": self.global_step}, self.hparams.checkpoint_dir / f"checkpoint_{update}.pt")

    def _load_checkpoint(self, step: int):
        ck = torch.load(self.hparams.checkpoint_dir / f"checkpoint_{step}.pt", map_location=self.device,
                        weights_only=True)
        self.agent.load_state_dict(ck["agent"])
        self.optimizer.load_state_dict(ck["optimizer"])
        self.update = ck["update"] + 1
        self.global_step = ck["global_step"]
