"""The Coach (blokus_rl/alphazero/trainer.py:27-376), self-play half on the MI355X engine.

* `_self_play(temperature)` — the reference episode (trainer.py:92-137) on the drop-in
  Game/MCTS/NNet classes, with the reference's np.random calls in the reference's order
  (Dirichlet on the first ply, np.random.choice per ply), so a seeded run is the reference's.
* `self_play_batched(games)` — the same episode for `games_per_gpu` games at once on the batched
  engine (alphazero/selfplay.py): the throughput path.
* `train()` iterations (trainer.py:138-221), every stage on the device:
  batched self-play -> packed replay rows (all-gathered over ranks, written as a binary shard
  data/train/iteration_i/shard_<rank>.bkrp, optionally also in the reference's pickled layout)
  -> DeviceReplay window -> Learner epochs (bk_replay_batch + HIP policy loss, DDP over RCCL)
  -> batched arena compare of the new net against the previous one (T=0 MCTS players) -> Elo
  update (trainer.py:322-334) -> checkpoint. Tensorboard/video logging are not reproduced.
"""
from __future__ import annotations

from pathlib import Path
from pickle import Pickler

import numpy as np
import torch

import copy

import torch.distributed as dist

from .. import replay as rp
from .. import replay_io as rio
from ..colossumrl import ColosseumBlokusGameWrapper
from ..neural_network import BlokusNNetWrapper
from .batched_arena import ArenaSeat, BatchedArena
from .learner import DeviceReplay, Learner
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
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        self.replay = None
        self.learner = None
        self.pnet_model = None
        self.history: list[dict] = []

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

    def self_play_packed(self, games: int | None = None, max_plies: int = 200, seed: int = 0):
        """`games` complete episodes -> packed replay rows (uint8 [E, stride], cap) on the device."""
        G = games or self.hparams.games_per_gpu
        dt = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[self.hparams.nn_dtype]
        sp = SelfPlay(self.game.engine, self.nnet.model, G, num_sims=self.hparams.num_mcts_sims,
                      cpuct=self.hparams.cpuct, temperature=self.hparams.temperature, seed=seed, nn_dtype=dt)
        sp.run(max_plies)
        ex = sp.examples()
        if ex is None:
            return torch.zeros((0, rp.stride_of(64)), dtype=torch.uint8, device=self.game.device), 64
        return rp.pack(ex.states, ex.ids, ex.pi, ex.k, ex.z)

    # ------------------------------------------------------------------ device iteration
    def _compute_new_elo(self, agent_elo: float, opponent_elo: float, agent_score: float) -> float:
        """trainer.py:322-334."""
        expected = 1 / (1 + 10 ** ((opponent_elo - agent_elo) / 400))
        return agent_elo + self.hparams.elo_convert_rate * (1 - expected) * agent_score

    def arena_compare(self, opponent_model=None, games: int | None = None):
        """_arena_compare (trainer.py:222-271): the agent's net against P-1 seats of the
        previous net (DumbNet/None = the uninformed MCTS opponent), batched, T=0 moves."""
        P = self.game.number_of_players
        sims = self.hparams.num_mcts_sims
        seats = [ArenaSeat(self.nnet.model.eval(), sims)] + [ArenaSeat(opponent_model, sims) for _ in range(P - 1)]
        arena = BatchedArena(self.game.engine, seats, cpuct=1.0)
        scores, _, _ = arena.play(games or self.hparams.compare_arena_games, permute=self.hparams.permute)
        return scores

    def run_iteration_device(self, games: int | None = None, seed: int | None = None, save: bool = True,
                             arena_games: int | None = None):
        """One policy-improvement iteration on the device path; returns its summary."""
        eng = self.game.engine
        seed = self.iteration * 1000 + self.rank if seed is None else seed
        rows, cap = self.self_play_packed(games, seed=seed)
        if save:
            rio.write_shard(rio.shard_path(self.hparams.data_dir, self.iteration, self.rank), rows, cap,
                            eng.N, eng.P, self.iteration)
            if getattr(self.hparams, "save_legacy_examples", False):
                self._save_train_examples(Path(self.hparams.data_dir) / f"iteration_{self.iteration}", self.rank,
                                          rio.packed_to_legacy(rows, cap, eng))
        if self.world > 1:
            rows, cap = rp.all_gather_packed(rows, cap)
        if self.replay is None:
            self.replay = DeviceReplay(eng, cap=max(1024, cap),
                                       history=self.hparams.num_iters_for_train_examples_history)
        self.replay.add_packed(rows, cap)
        # the previous net (the reference saves temp.pth.tar before training and loads it as pnet)
        self.pnet_model = copy.deepcopy(self.nnet.model).eval()
        if self.learner is None:
            self.learner = Learner(self.nnet.model, batch_size=self.hparams.batch_size, seed=self.hparams.seed,
                                   optimizer=self.nnet.optimizer)
        loss = self.learner.train_epochs(self.replay, self.hparams.epochs)
        self.train_epoch += self.hparams.epochs
        self.nnet.latest_loss = loss
        self.nnet.mean_loss.update(loss)
        self.nnet._infer = None
        summary = {"iteration": self.iteration, "examples": int(rows.shape[0]), "replay_rows": len(self.replay),
                   "loss": loss}
        if arena_games != 0:
            scores = self.arena_compare(self.pnet_model, arena_games)
            old = self.nnet.elo  # pnet is loaded from the pre-training checkpoint: same Elo (trainer.py:191-202)
            self.nnet.elo = self._compute_new_elo(old, old, float(scores[0]))
            summary.update(arena_scores=scores.tolist(), elo=self.nnet.elo)
        if save and self.rank == 0:
            self.nnet.save_checkpoint(filename=self.nnet.get_checkpoint_file(self.iteration))
        self.history.append(summary)
        return summary

    # ------------------------------------------------------------------ legacy-layout iterations
    def _save_train_examples(self, save_dir: Path, episode: int, examples):
        save_dir.mkdir(parents=True, exist_ok=True)
        with open(save_dir / self.nnet.get_data_file(episode), "wb+") as f:
            Pickler(f).dump(examples)

    def _load_examples(self):
        """Legacy `.examples` files of the last history window, through the allow-list unpickler
        (replay_io.load_legacy): the directory may hold files this process did not write."""
        data = []
        files = sorted(Path(self.hparams.data_dir).rglob("*.examples"))
        for fp in files[-self.hparams.num_iters_for_train_examples_history:]:
            data.extend(rio.load_legacy(fp))
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
        return self.run_iteration_device(self.hparams.num_eps)

    def train(self):
        for _ in range(self.hparams.num_iters):
            self.iteration += 1
            self._run_iteration()
