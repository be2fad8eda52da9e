"""The Coach (blokus_rl/alphazero/trainer.py:27-376), self-play half on the MI355X engine.

* `_self_play(temperature)` — the reference episode (trainer.py:92-137) on the drop-in
  Game/MCTS/NNet classes, with the reference's np.random calls in the reference's order
  (Dirichlet on the first ply, np.random.choice per ply), so a seeded run is the reference's.
* `self_play_batched(games)` — the same episode for `games_per_gpu` games at once on the batched
  engine (alphazero/selfplay.py): the throughput path.
* `train()` iterations: self-play -> pickled examples in the reference layout
  (data/train/iteration_i/checkpoint_e.examples, trainer.py:287-292) -> epochs of train_step ->
  checkpoint. Arena/Elo/video logging are outside the accelerated path.
"""
from __future__ import annotations

from pathlib import Path
from pickle import Pickler, Unpickler

import numpy as np
import torch

from ..colossumrl import ColosseumBlokusGameWrapper
from ..neural_network import BlokusNNetWrapper
from .mcts import MCTS
from .selfplay import SelfPlay


class AlphaZeroTrainer:
    def __init__(self, hparams):
        self.hparams = hparams
        self.device = "cuda" if torch.cuda.is_available() and hparams.cuda else "cpu"
        self.game = ColosseumBlokusGameWrapper(hparams)
        self.nnet = BlokusNNetWrapper(self.game, hparams, self.device)
        self.iteration = 0
        self.train_epoch = 0

    # ------------------------------------------------------------------ reference episode
    def _self_play(self, temperature):
        s, current_player = self.game.get_init_board()
        tree = MCTS(self.game, self.nnet)
        data = []
        scores = self.game.get_game_ended(s)
        root, alpha, weight = True, 1, 0.25
        while scores is None:
            for _ in range(self.hparams.num_mcts_sims):
                tree.simulate(s, current_player, cpuct=self.hparams.cpuct)
            dist = tree.get_distribution(s, temperature=temperature)
            if root:
                noise = np.random.dirichlet(np.array(alpha * np.ones_like(dist[:, 1].astype(np.float32))))
                dist[:, 1] = dist[:, 1] * (1 - weight) + noise * weight
                root = False
            obs, mask = self.game.get_observation(s, current_player)
            data.append([obs, mask, dist[:, 1].astype(np.float32), None])
            idx = np.random.choice(len(dist), p=dist[:, 1].astype(np.float32))
            a = dist[idx, 0][0]
            s, current_player = self.game.get_next_state(s, current_player, a)
            scores = self.game.get_game_ended(s)
        for item in data:
            item[-1] = scores
        return data

    # ------------------------------------------------------------------ batched episodes
    def self_play_batched(self, games: int | None = None, max_plies: int = 200, seed: int = 0):
        """`games` complete episodes on the batched engine; returns reference-format examples
        [obs, mask(float64[A]), pi(float32[K]), z(float64[P])]."""
        G = games or self.hparams.games_per_gpu
        dt = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[self.hparams.nn_dtype]
        sp = SelfPlay(self.game.engine, self.nnet.model, G, num_sims=self.hparams.num_mcts_sims,
                      cpuct=self.hparams.cpuct, temperature=self.hparams.temperature, seed=seed, nn_dtype=dt)
        sp.run(max_plies)
        ex = sp.examples()
        if ex is None:
            return []
        eng = self.game.engine
        obs = eng.observe(ex.states).cpu().numpy()
        masks, _ = eng.legal_mask(ex.states)
        bits = eng.unpack_mask(masks).cpu().numpy().astype(np.float64)
        k, pi, z = ex.k.cpu().numpy(), ex.pi.cpu().numpy(), ex.z.cpu().numpy().astype(np.float64)
        return [[obs[i], bits[i], pi[i, : k[i]].copy(), z[i]] for i in range(len(ex))]

    # ------------------------------------------------------------------ iterations
    def _save_train_examples(self, save_dir: Path, episode: int, examples):
        save_dir.mkdir(parents=True, exist_ok=True)
        with open(save_dir / self.nnet.get_data_file(episode), "wb+") as f:
            Pickler(f).dump(examples)

    def _load_examples(self):
        data = []
        files = sorted(Path(self.hparams.data_dir).rglob("*.examples"))
        for fp in files[-self.hparams.num_iters_for_train_examples_history:]:
            with open(fp, "rb") as f:  # files this trainer wrote itself
                data.extend(Unpickler(f).load())
        return data

    def _train_epochs(self, data):
        from torch.nn.utils.rnn import pad_sequence

        bs = self.hparams.batch_size
        losses = []
        for _ in range(self.hparams.epochs):
            self.train_epoch += 1
            perm = np.random.permutation(len(data))
            for i in range(0, len(perm), bs):
                items = [data[j] for j in perm[i:i + bs]]
                batch = {
                    "observation": torch.stack([torch.from_numpy(np.asarray(x[0])).float() for x in items]),
                    "mask": torch.stack([torch.from_numpy(x[1]).bool() for x in items]),
                    "prob": pad_sequence([torch.from_numpy(x[2]).float() for x in items], batch_first=True),
                    "score": torch.stack([torch.from_numpy(np.asarray(x[3])).float() for x in items]),
                }
                losses.append(self.nnet.train_step(batch))
        return float(np.mean(losses)) if losses else 0.0

    def _run_iteration(self):
        save_dir = Path(self.hparams.data_dir) / f"iteration_{self.iteration}"
        examples = self.self_play_batched(self.hparams.num_eps)
        self._save_train_examples(save_dir, 0, examples)
        loss = self._train_epochs(self._load_examples())
        self.nnet.save_checkpoint(filename=self.nnet.get_checkpoint_file(self.iteration))
        return loss

    def train(self):
        for _ in range(self.hparams.num_iters):
            self.iteration += 1
            self._run_iteration()
