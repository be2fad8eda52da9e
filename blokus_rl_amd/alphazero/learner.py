"""The learner half of the AlphaZero iteration on the device.

Reference path (blokus_rl/alphazero/trainer.py:158-186, neural_network.py:52-85, :138-157,
alphazero/dataset.py:12-54): pickled examples [obs, f64 mask, f32 pi, f64 z] -> a DataLoader
(shuffle=True, batch_size, pad_sequence collate) -> per batch: host->device copy, forward,
compute_loss with a per-sample Python loop of masked_select + log_softmax, Adam step.

Here the examples stay in HBM as packed replay rows (replay.py), the batch is decoded on the
device by bk_replay_batch (observation planes + sparse pi + z in one launch), and the policy
term of compute_loss is the bk_policy_loss / bk_policy_loss_grad kernel pair over the sparse pi
(only the K legal logits per row are read). The value term, the optimiser (Adam with the
reference's lr / weight_decay) and the net stay in PyTorch-ROCm. With torch.distributed
initialised the model is wrapped in DistributedDataParallel (RCCL all-reduce of gradient
buckets, overlapped with backward) and each rank trains on its shard of the shared epoch
permutation — weak scaling over ranks, global batch = batch_size x world.
"""
from __future__ import annotations

import ctypes
from collections import deque

import torch
import torch.distributed as dist

from ..engine import _check, _ptr, _stream, load_library
from .. import replay as rp


class PolicyLoss(torch.autograd.Function):
    """mean_b( -sum_j pi_bj * log_softmax(x_b[ids_b])_j ) over the rows' legal ids (HIP)."""

    @staticmethod
    def forward(ctx, x, ids, pi, k):
        lib = load_library()
        x = x.float().contiguous()
        B = x.shape[0]
        cap = ids.shape[1]
        loss = torch.empty(B, dtype=torch.float32, device=x.device)
        lse = torch.empty(B, dtype=torch.float32, device=x.device)
        _check(lib.bk_policy_loss(_ptr(x), x.shape[1], _ptr(ids), _ptr(pi), _ptr(k), cap, B, _ptr(loss), _ptr(lse),
                                  _stream(x.device)))
        ctx.save_for_backward(x, ids, pi, k, lse)
        return loss.sum() / max(B, 1)

    @staticmethod
    def backward(ctx, g):
        lib = load_library()
        x, ids, pi, k, lse = ctx.saved_tensors
        B = x.shape[0]
        grad = torch.zeros_like(x)
        g = g.float().contiguous()
        _check(lib.bk_policy_loss_grad(_ptr(x), x.shape[1], _ptr(ids), _ptr(pi), _ptr(k), ids.shape[1], B, _ptr(lse),
                                       ctypes.c_float(1.0 / max(B, 1)), _ptr(g), _ptr(grad), grad.shape[1],
                                       _stream(x.device)))
        return grad, None, None, None


def policy_loss(x: torch.Tensor, ids: torch.Tensor, pi: torch.Tensor, k: torch.Tensor) -> torch.Tensor:
    for t, dt in ((ids, torch.int16), (pi, torch.float32), (k, torch.int32)):
        if t.dtype != dt or not t.is_contiguous():
            raise TypeError(f"policy_loss expects contiguous {dt}, got {t.dtype}")
    return PolicyLoss.apply(x, ids, pi, k)


_IDENT: dict = {}


def sparse_policy_loss(xs: torch.Tensor, pi: torch.Tensor, k: torch.Tensor) -> torch.Tensor:
    """policy_loss on logits already gathered at the rows' legal ids (xs [B, cap]: column j = the
    logit of ids[b][j], SparsePolicyLinear): the same kernels with the identity id map."""
    B, cap = xs.shape
    key = (xs.device, B, cap)
    ident = _IDENT.get(key)
    if ident is None:
        ident = _IDENT[key] = torch.arange(cap, dtype=torch.int16, device=xs.device).expand(B, cap).contiguous()
    return PolicyLoss.apply(xs, ident, pi, k)


def alphazero_loss(p_pred, v_pred, batch, policy_fn=policy_loss):
    """compute_loss (neural_network.py:138-157): policy cross-entropy over the legal ids + value
    MSE `(v_pred.squeeze() - z).pow(2).mean()`."""
    v_loss = (v_pred.squeeze() - batch["score"]).pow(2).mean()
    return policy_fn(p_pred, batch["ids"], batch["pi"], batch["k"]) + v_loss


class DeviceReplay:
    """Packed replay rows resident in HBM, kept for the last `history` iterations (the
    reference's num_iters_for_train_examples_history window over its .examples files,
    dataset.py:29-36)."""

    def __init__(self, engine, cap: int = 1024, history: int = 20):
        if cap % 64:
            raise ValueError("cap must be a multiple of 64")
        self.engine, self.cap, self.history = engine, cap, history
        self.stride = rp.stride_of(cap)
        self._chunks: deque[torch.Tensor] = deque()
        self._rows: torch.Tensor | None = None

    def add_packed(self, buf: torch.Tensor, cap: int):
        """Rows of one iteration (packed at any cap) -> the window (re-packed to this cap)."""
        if cap != self.cap:
            u = rp.unpack(buf, cap, self.engine.P)
            if buf.shape[0] and int(u["k"].max()) > self.cap:
                raise ValueError(f"an example has K={int(u['k'].max())} > replay cap {self.cap}")
            buf, _ = rp.pack(u["states"], u["ids"].to(torch.int32), u["pi"], u["k"], u["z"], u["player"],
                             cap=self.cap)
        self._chunks.append(buf.to(self.engine.device).contiguous())
        while len(self._chunks) > self.history:
            self._chunks.popleft()
        self._rows = None

    def add_examples(self, ex):
        """A SelfPlay.examples() set (states, ids, pi, k, z, player)."""
        buf, cap = rp.pack(ex.states, ex.ids, ex.pi, ex.k, ex.z, getattr(ex, "player", None))
        self.add_packed(buf, cap)

    @property
    def rows(self) -> torch.Tensor:
        if self._rows is None:
            self._rows = (torch.cat(list(self._chunks)) if self._chunks else
                          torch.zeros((0, self.stride), dtype=torch.uint8, device=self.engine.device))
        return self._rows

    def __len__(self):
        return sum(c.shape[0] for c in self._chunks)

    def batch(self, index: torch.Tensor) -> dict:
        return self.engine.replay_batch(self.rows, self.cap, index)


class Learner:
    """Adam on the reference's net with the device batch path; DDP when a process group is up."""

    def __init__(self, model: torch.nn.Module, lr: float = 1e-3, weight_decay: float = 1e-4, batch_size: int = 64,
                 seed: int = 0, policy_fn=policy_loss, group=None, optimizer: torch.optim.Optimizer | None = None,
                 device_path: bool | str = "auto"):
        """device_path: train the ResNet on train_conv's device path (tower convs on bk_conv_x3,
        channels_last, PyTorch batch norm; switched in place) — True, False, or "auto" = on a GPU
        at batch_size >= 256 (the large batches where the fp32 convolutions dominate a step)."""
        self.model = model
        self.batch_size = batch_size
        on_gpu = next(model.parameters()).is_cuda
        if device_path == "auto":
            device_path = on_gpu and batch_size >= 256
        self.device_path = bool(device_path)
        if self.device_path:
            from .train_conv import TrainResNet, prepare_model
            prepare_model(model)
            # the policy Linear at the batch's legal ids only (trainfc.hip), with the reference loss
            self.sparse_head = isinstance(model, TrainResNet) and policy_fn is policy_loss
        else:
            self.sparse_head = False
        self.policy_fn = policy_fn
        self.group = group
        up = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if up else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        self.net = model
        if up:  # DDP whenever a group is up (at world size 1 too: the RCCL path on a one-GPU box)
            dev = next(model.parameters()).device
            self.net = torch.nn.parallel.DistributedDataParallel(
                model, device_ids=[dev.index] if dev.type == "cuda" else None, process_group=group)
        self.optimizer = optimizer or torch.optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay)
        self.gen = torch.Generator().manual_seed(seed)
        self.steps = 0

    def train_step(self, batch: dict) -> torch.Tensor:
        """train_step (neural_network.py:52-85) without the host sync: returns the loss tensor."""
        self.net.train()
        obs = batch["observation"]
        if self.device_path:
            obs = obs.contiguous(memory_format=torch.channels_last)
        if self.sparse_head:
            xs, v_pred = self.net(obs, ids=batch["ids"], k=batch["k"])
            loss = sparse_policy_loss(xs, batch["pi"], batch["k"]) + (v_pred.squeeze() - batch["score"]).pow(2).mean()
        else:
            p_pred, v_pred = self.net(obs)
            loss = alphazero_loss(p_pred, v_pred, batch, self.policy_fn)
        self.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        self.optimizer.step()
        self.steps += 1
        return loss.detach()

    def epoch_indices(self, n: int) -> torch.Tensor:
        """This rank's shard of one shuffled epoch (DataLoader(shuffle=True), split like
        DistributedSampler without padding: every rank gets the same number of rows)."""
        perm = torch.randperm(n, generator=self.gen)
        per = n // self.world if self.world > 1 else n
        return perm[self.rank * per:(self.rank + 1) * per] if self.world > 1 else perm

    def train_epochs(self, replay, epochs: int = 1, batch_fn=None) -> float:
        """`epochs` passes over the replay window; mean loss over all steps (one host sync)."""
        batch_fn = batch_fn or replay.batch
        total, count = None, 0
        dev = next(self.model.parameters()).device
        for _ in range(epochs):
            idx = self.epoch_indices(len(replay)).to(dev)
            for i in range(0, idx.shape[0], self.batch_size):
                loss = self.train_step(batch_fn(idx[i:i + self.batch_size]))
                total = loss if total is None else total + loss
                count += 1
        return float(total / count) if count else 0.0
