"""PPO agents (blokus_rl/ppo/agent.py:12-254) with the reference's state_dict layout, so its
checkpoints load unchanged. The legal-move filter runs on the device: FilterLegalMoves takes the
vector env's bitmask words and applies the reference's rule in one kernel (bk_filter_legal),
instead of building a dense mask in a Python loop over `ai_possible_indexes`."""
from __future__ import annotations

import numpy as np
import torch
from torch import nn
from torch.distributions.categorical import Categorical

from ..engine import _check, _ptr, _stream, load_library


def layer_init(layer: nn.Linear, std=float(np.sqrt(2)), bias_const=0.0) -> nn.Linear:
    """agent.py:12-24: orthogonal weights, constant bias."""
    torch.nn.init.orthogonal_(layer.weight, std)
    torch.nn.init.constant_(layer.bias, bias_const)
    return layer


def ids_to_mask_words(possible_moves, A: int, device) -> torch.Tensor:
    """A list of legal-id lists (the reference's `ai_possible_indexes`) -> [E, ceil(A/64)] words."""
    E, W = len(possible_moves), (A + 63) // 64
    bits = np.zeros((E, W * 64), dtype=np.uint8)
    for i, m in enumerate(possible_moves):
        bits[i, np.asarray(m, dtype=np.int64)] = 1
    words = (bits.reshape(E, W, 64).astype(np.uint64) << np.arange(64, dtype=np.uint64)).sum(axis=2, dtype=np.uint64)
    return torch.from_numpy(words.view(np.int64)).to(device)


class FilterLegalMoves(nn.Module):
    """agent.py:27-42: x * mask, every resulting 0 -> -1e9 (a legal logit of exactly 0 too)."""

    def forward(self, x, possible_moves):
        if not isinstance(possible_moves, torch.Tensor):
            possible_moves = ids_to_mask_words(possible_moves, x.shape[1], x.device)
        if x.device.type != "cuda":
            raise RuntimeError("FilterLegalMoves runs on the HIP device (bk_filter_legal)")
        x = x.float().contiguous()
        words = possible_moves.contiguous()
        out = torch.empty_like(x)
        _check(load_library().bk_filter_legal(_ptr(x), x.shape[0], x.shape[1], _ptr(words), words.shape[1],
                                              _ptr(out), _stream(x.device)))
        if torch.is_grad_enabled() and x.requires_grad:
            # the reference's op is differentiable w.r.t. the kept logits (x * mask): route the
            # gradient through where the output kept x
            keep = out != -1e9
            return torch.where(keep, x, out.detach())
        return out


class MLP(nn.Module):
    """agent.py:163-196: 3 hidden ReLU layers (h, 2h, h) with dropout, orthogonal init."""

    def __init__(self, input_dim, hidden_dim, output_dim, dropout=0.1, std=0.01):
        super().__init__()
        dims = [input_dim, hidden_dim, hidden_dim * 2, hidden_dim]
        layers: list[nn.Module] = []
        for a, b in zip(dims[:-1], dims[1:]):
            layers += [layer_init(nn.Linear(a, b)), nn.Dropout(dropout), nn.ReLU()]
        layers.append(layer_init(nn.Linear(hidden_dim, output_dim), std))
        self.net = nn.Sequential(*layers)
        self.filter_legal_moves = FilterLegalMoves()

    def forward(self, x, possible_moves=None):
        x = self.net(x)
        return x if possible_moves is None else self.filter_legal_moves(x, possible_moves)


class ConvBlock(nn.Module):
    """agent.py:45-103: n_layers x (conv, dropout, ReLU) on a 1-channel board."""

    def __init__(self, in_channels, out_channels, n_layers=4, kernel_size=3, stride=1, padding=1, dropout=0.1):
        super().__init__()
        if n_layers < 1:
            raise ValueError("Number of layers must be at least 1")
        layers: list[nn.Module] = []
        c = in_channels
        for _ in range(n_layers):
            layers += [nn.Conv2d(c, out_channels, kernel_size, stride=stride, padding=padding), nn.Dropout(dropout),
                       nn.ReLU()]
            c = out_channels
        self.conv_block = nn.Sequential(*layers)

    def forward(self, x):
        return self.conv_block(x.unsqueeze(1))


class _ActorCritic(nn.Module):
    def features(self, x):
        raise NotImplementedError

    def forward(self, x, possible_moves=None):
        return self.actor(self.features(x), possible_moves)

    def get_value(self, x):
        return self.critic(self.features(x))

    def get_action_and_value(self, x, action=None, possible_moves=None):
        h = self.features(x)
        probs = Categorical(logits=self.actor(h, possible_moves))
        if action is None:
            action = probs.sample()
        return action, probs.log_prob(action), probs.entropy(), self.critic(h)


class CnnAgent(_ActorCritic):
    """agent.py:106-160."""

    def __init__(self, obs_shape, n_actions: int, hparams):
        super().__init__()
        self.input_dim = tuple(obs_shape)
        self.board_dim = int(np.prod(obs_shape))
        self.output_dim = n_actions
        self.d_model = hparams.d_model
        self.conv_block = ConvBlock(1, self.d_model, hparams.cnn_layers, hparams.cnn_kernel_size, hparams.cnn_stride,
                                    hparams.cnn_padding, hparams.cnn_dropout)
        flat = self.d_model * self.board_dim
        self.actor = MLP(flat, self.d_model, n_actions, hparams.dropout, std=0.01)
        self.critic = MLP(flat, self.d_model, 1, hparams.dropout, std=1.0)

    def features(self, x):
        h = self.conv_block(x)
        return h.reshape(h.size(0), -1)  # (c, h, w) order whatever the conv layout (channels_last too)


class MlpAgent(_ActorCritic):
    """agent.py:199-248."""

    def __init__(self, obs_shape, n_actions: int, hparams):
        super().__init__()
        self.input_dim = int(np.prod(obs_shape))
        self.output_dim = n_actions
        self.d_model = hparams.d_model
        self.actor = MLP(self.input_dim, self.d_model, n_actions, hparams.dropout, std=0.01)
        self.critic = MLP(self.input_dim, self.d_model, 1, hparams.dropout, std=1.0)

    def features(self, x):
        if x.ndim == 1:
            return x.unsqueeze(0)
        if x.ndim >= 3:
            return x.reshape(-1, self.input_dim)
        return x


def get_agent(agent: str):
    return {"mlp": MlpAgent, "cnn": CnnAgent}[agent]
