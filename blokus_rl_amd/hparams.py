"""Hyper-parameters consumed by the hot path, with the reference's field names and YAML keys
(blokus_rl/hparams.py:11-290) so its config files load unchanged. Only the fields the
self-play path reads are typed here; every other key of a reference YAML is accepted and kept
as an attribute. New keys: `max_piece_cells`, `games_per_gpu`, `nn_dtype`."""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path

import yaml


@dataclass
class AlphaZeroHparams:
    # board (hparams.py:192-196)
    board_size: int = 20
    number_of_players: int = 4
    states_dir: Path = Path("states")
    max_piece_cells: int = 5
    # model (hparams.py:199-213)
    model_type: str = "resnet"
    num_res_blocks: int = 5
    lr: float = 0.001
    dropout: float = 0.3
    epochs: int = 10
    batch_size: int = 64
    num_channels: int = 128
    linear_dim: int = 128
    weight_decay: float = 1e-4
    # self-play / search (hparams.py:216-248)
    num_iters: int = 1000
    num_eps: int = 100
    num_mcts_sims: int = 100
    arena_num_mcts_sims: int = 50
    compare_arena_games: int = 24
    permute: bool = True
    cpuct: int = 1
    elo_convert_rate: int = 20
    temperature: float = 1.0
    # checkpoints / data (hparams.py:14-40, 251-265)
    checkpoint_dir: Path = Path("models/checkpoints")
    data_dir: Path = Path("data/train")
    val_data_dir: Path = Path("data/valid")
    log_dir: Path = Path("models/logs")
    load_checkpoint_step: int | None = None
    best_model_name: str = "best.pth.tar"
    temp_model_name: str = "temp.pth.tar"
    num_iters_for_train_examples_history: int = 20
    skip_first_self_play: bool = False
    opponent_type: str = "uninformed"
    experiment_name: str = "blokus"
    cuda: bool = True
    seed: int = 42
    capture_video: bool = False
    verbose: bool = False
    # MI355X engine
    games_per_gpu: int = 256
    nn_dtype: str = "fp32"
    extra: dict = field(default_factory=dict)

    def __post_init__(self):
        for k in ("states_dir", "checkpoint_dir", "data_dir", "val_data_dir", "log_dir"):
            setattr(self, k, Path(getattr(self, k)))

    @classmethod
    def from_dict(cls, d: dict) -> "AlphaZeroHparams":
        known = {f for f in cls.__dataclass_fields__}
        hp = cls(**{k: v for k, v in d.items() if k in known})
        hp.extra = {k: v for k, v in d.items() if k not in known}
        for k, v in hp.extra.items():
            setattr(hp, k, v)
        return hp


def load_hparams(hparam_fp: Path | str | None = None, algorithm: str = "alphazero"):
    """hparams.py:284-290 (returns an instance; the reference returns the class when no file
    is given, which works there only because dataclass defaults are class attributes)."""
    if algorithm != "alphazero":
        raise ValueError("this engine accelerates the alphazero path; PPO uses blokus_rl_amd.vector_env")
    if hparam_fp is None:
        return AlphaZeroHparams()
    with open(hparam_fp, "r", encoding="utf-8") as f:
        return AlphaZeroHparams.from_dict(yaml.safe_load(f) or {})
