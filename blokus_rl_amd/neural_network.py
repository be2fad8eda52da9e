"""Drop-in `BlokusNNetWrapper` (blokus_rl/neural_network.py:11-210).

Keeps the reference API — predict(x, mask) -> (p over the legal ids, v), get_valid_dist,
compute_loss, train_step, save/load_checkpoint with the same checkpoint keys — and adds
`predict_batch(obs)`, the device-side leaf evaluation the batched MCTS uses: the BN-folded
inference form of the net over a [G, 2P, N, N] batch, returning log-probabilities over all A
ids and values (the masked softmax then runs inside k_expand_backup).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

from .nets import build_model, inference_model


class AverageMeter:
    def __init__(self):
        self.val = self.avg = self.sum = 0.0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


class BlokusNNetWrapper:
    def __init__(self, game, hparams, device: str | torch.device = "cuda", model_type: str | None = None):
        self.game = game
        self.hparams = hparams
        self.device = torch.device(device)
        self.model_type = model_type or hparams.model_type
        self.model = build_model(self.model_type, game.board_size, game.number_of_players, game.get_action_size(),
                                 num_res_blocks=getattr(hparams, "num_res_blocks", 5),
                                 num_channels=getattr(hparams, "num_channels", 128),
                                 linear_dim=getattr(hparams, "linear_dim", 128),
                                 dropout=getattr(hparams, "dropout", 0.3)).to(self.device)
        self.elo = 1000
        self.latest_loss = 0
        self.mean_loss = AverageMeter()
        self._infer = None
        self.optimizer = None
        if len(list(self.model.parameters())) > 0:
            self.optimizer = torch.optim.Adam(self.model.parameters(), lr=hparams.lr,
                                              weight_decay=hparams.weight_decay)

    @staticmethod
    def get_checkpoint_file(iteration: int):
        return "checkpoint_" + str(iteration) + ".pth.tar"

    @staticmethod
    def get_data_file(iteration: int):
        return "checkpoint_" + str(iteration) + ".examples"

    # ------------------------------------------------------------------ inference
    @torch.inference_mode()
    def predict(self, x, mask):
        """neural_network.py:92-110: batch-1 forward, p = softmax over the legal logits."""
        self.model.eval()
        x = torch.from_numpy(np.asarray(x)).float().to(self.device).unsqueeze(0)
        mask = torch.from_numpy(np.asarray(mask)).bool().to(self.device)
        p_logits, v = self.model(x)
        p = self.get_valid_dist(mask, p_logits[0])
        return p.cpu().numpy().squeeze(), v.cpu().numpy().squeeze()

    @torch.inference_mode()
    def predict_batch(self, obs: torch.Tensor, dtype: torch.dtype = torch.float32):
        """Leaf batch on the device: obs [G, 2P, N, N] f32 -> (logp [G, A] f32, v [G, P] f32)."""
        if self._infer is None:
            self._infer = inference_model(self.model).to(memory_format=torch.channels_last)
        obs = obs.contiguous(memory_format=torch.channels_last)
        if dtype != torch.float32:
            with torch.autocast("cuda", dtype=dtype):
                lp, v = self._infer(obs)
        else:
            lp, v = self._infer(obs)
        return lp.float().contiguous(), v.float().contiguous()

    def get_valid_dist(self, mask, logits, log_softmax=False):
        """neural_network.py:159-173."""
        dist = F.log_softmax(torch.masked_select(logits, mask), dim=-1)
        return dist if log_softmax else torch.exp(dist)

    # ------------------------------------------------------------------ training
    def compute_loss(self, masks, prediction, target):
        """neural_network.py:138-157, vectorised: v MSE + mean over samples of
        -sum(pi * log_softmax(logits[legal])) with pi padded to the longest K."""
        p_pred, v_pred = prediction
        p_gt, v_gt = target
        v_loss = (v_pred.squeeze() - v_gt).pow(2).mean()
        masks = masks.bool()
        lsm = F.log_softmax(p_pred.masked_fill(~masks, float("-inf")), dim=-1)
        pos = torch.cumsum(masks.long(), dim=1) - 1  # rank of a legal id among the row's legal ids
        pos = pos.clamp(min=0, max=p_gt.shape[1] - 1)
        gt = torch.gather(p_gt, 1, pos)
        p_loss = -(torch.where(masks, gt * lsm, torch.zeros_like(lsm))).sum() / masks.size(0)
        return p_loss + v_loss

    def train_step(self, batch):
        self.model.train()
        self._infer = None
        batch = {k: v.to(self.device) for k, v in batch.items()}
        p_pred, v_pred = self.model(batch["observation"])
        loss = self.compute_loss(batch["mask"], (p_pred, v_pred), (batch["prob"], batch["score"]))
        self.optimizer.zero_grad()
        loss.backward()
        self.optimizer.step()
        self.latest_loss = loss.item()
        self.mean_loss.update(self.latest_loss)
        return loss.item()

    # ------------------------------------------------------------------ checkpoints
    def save_checkpoint(self, filename: str = "checkpoint.pth.tar"):
        path = Path(self.hparams.checkpoint_dir) / filename
        path.parent.mkdir(parents=True, exist_ok=True)
        torch.save({"nnet": self.model.state_dict(),
                    "optimizer": self.optimizer.state_dict() if self.optimizer else {},
                    "mean_loss": self.mean_loss.avg, "latest_loss": self.latest_loss, "elo": self.elo}, path)

    def load_checkpoint(self, iteration: int):
        if self.hparams.load_checkpoint_step is None:
            return
        name = self.get_checkpoint_file(iteration)
        if (Path(self.hparams.checkpoint_dir) / self.hparams.best_model_name).exists():
            name = self.hparams.best_model_name
        self._load_checkpoint(name)

    def _load_checkpoint(self, filename: str = "checkpoint.pth.tar"):
        path = Path(self.hparams.checkpoint_dir) / filename
        assert path.exists(), f"Model path doesn't exist {path}"
        ck = torch.load(path, map_location=self.device, weights_only=True)
        self.model.load_state_dict(ck["nnet"])
        if self.optimizer and ck.get("optimizer"):
            self.optimizer.load_state_dict(ck["optimizer"])
        self.mean_loss.update(ck["mean_loss"])
        self.latest_loss = ck["latest_loss"]
        self.elo = ck["elo"]
        self._infer = None
