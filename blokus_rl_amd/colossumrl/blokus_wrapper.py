"""Drop-in `ColosseumBlokusGameWrapper` (blokus_rl/colossumrl/blokus_wrapper.py:21-324) backed
by the HIP engine instead of colosseumrl.

Same method names, argument meaning and return conventions as the reference:
  get_init_board() -> (state, 0); get_next_state(state, player, id|str) -> (state', player');
  get_valid_moves(state, player) -> float64[A]; get_observation(state, player) -> (obs, mask);
  get_game_ended(state) -> None | float64[P] (-1 / 3 / 1); string_representation(state) -> int
  (board-only key); get_action_size / get_observation_size / get_board_size /
  get_number_of_players; get_sample_move; get_valid_actions_for_human_player; display; render.
A state is a 384-byte uint8 numpy array (the packed layout of include/blokus_engine.h), a value
the wrapper never mutates. Every rules computation runs on the GPU (batch 1 here; the batched
self-play path uses the same kernels at batch G). Unknown action strings raise KeyError as the
reference's dict lookup does (:130); an illegal id raises ValueError.
"""
from __future__ import annotations

import numpy as np
import torch

from ..engine import STATE_BYTES, W_FLAGS, W_HASH, W_TO_MOVE, Engine

PIECE_NAMES = ["I1", "I2", "I3", "V3", "I4", "L4", "T4", "S4", "O4", "F5", "I5", "L5", "N5", "P5", "T5",
               "U5", "V5", "W5", "X5", "Y5", "Z5"]
COLOURS = {0: (211, 211, 211), 1: (255, 0, 0), 2: (0, 0, 255), 3: (255, 255, 0), 4: (0, 128, 0)}


class ColosseumBlokusGameWrapper:
    def __init__(self, hparams, device: str | torch.device | None = None):
        self.hparams = hparams
        self.board_size = int(hparams.board_size)
        self.number_of_players = int(hparams.number_of_players)
        max_cells = int(getattr(hparams, "max_piece_cells", 5))
        self.engine = Engine(self.board_size, self.number_of_players, max_cells, device=device)
        self.device = self.engine.device
        tab = self.engine.action_table
        # action strings: "<piece>-<orientation>-<row>-<col>" of the placement's bounding box
        self.action_move_dict = {i: f"{PIECE_NAMES[p]}-{o}-{r}-{c}" for i, (p, o, r, c) in enumerate(tab)}
        self._move_action_dict = {v: k for k, v in self.action_move_dict.items()}
        self.starter_won = self.last_won = self.games_played = 0

    # ---------------------------------------------------------------- shape queries
    def get_board_size(self) -> tuple[int, int]:
        return (self.board_size, self.board_size)

    def get_action_size(self) -> int:
        return self.engine.A

    def get_observation_size(self) -> list[int]:
        return [self.number_of_players * 2, self.board_size, self.board_size]

    def get_number_of_players(self) -> int:
        return self.number_of_players

    # ---------------------------------------------------------------- device round trips
    def _dev(self, state: np.ndarray) -> torch.Tensor:
        return torch.from_numpy(np.ascontiguousarray(state, dtype=np.uint8).reshape(1, STATE_BYTES)).to(self.device)

    @staticmethod
    def _words(state: np.ndarray) -> np.ndarray:
        return np.asarray(state, dtype=np.uint8).view(np.int32)

    # ---------------------------------------------------------------- game API
    def get_init_board(self):
        st = self.engine.init_states(1)[0].cpu().numpy()
        return st, 0

    def get_next_state(self, current_state, current_player: int, action_id):
        """blokus_wrapper.py:89-106: id (or raw action string) -> (state', player')."""
        if isinstance(action_id, str):
            action_id = self._move_action_dict[action_id]  # KeyError like the reference
        a = torch.tensor([int(action_id)], dtype=torch.int32, device=self.device)
        out, nxt, status = self.engine.next_state(self._dev(current_state), a)
        if int(status[0]) != 0:
            raise ValueError(f"illegal action {action_id} for player {self.to_move(current_state)}")
        return out[0].cpu().numpy(), int(nxt[0])

    def get_valid_moves(self, current_state, current_player: int):
        """blokus_wrapper.py:108-132: float64[A], 1 at legal ids (current_player -1 -> to move)."""
        players = torch.tensor([int(current_player)], dtype=torch.int32, device=self.device)
        masks, _ = self.engine.legal_mask(self._dev(current_state), players)
        bits = np.unpackbits(masks.cpu().numpy().view(np.uint8), bitorder="little")[: self.engine.A]
        return bits.astype(np.float64)

    def get_observation(self, state, player: int):
        """blokus_wrapper.py:134-146: (canonical board [2P,N,N] f32, valid-move mask)."""
        obs = self.engine.observe(self._dev(state))[0].cpu().numpy()
        return obs, self.get_valid_moves(state, player)

    def get_valid_actions_for_human_player(self, state, player: int):
        ids = np.nonzero(self.get_valid_moves(state, player))[0]
        return [self.action_move_dict[int(i)] for i in ids] or [""]

    def get_game_ended(self, state):
        """blokus_wrapper.py:164-186: None while anyone can move, else -1 / 3 / 1 per player."""
        if not (int(self._words(state)[W_FLAGS]) & 1):
            return None
        _, scores = self.engine.game_ended(self._dev(state))
        return scores[0].cpu().numpy()

    def get_scores(self, winners):
        """blokus_wrapper.py:188-206 (unused by the training path)."""
        scores = np.ones(self.number_of_players) * -1
        if len(winners) == 1:
            scores[winners[0]] = 1
        else:
            for w in winners:
                scores[w] = 0
        return scores

    def string_representation(self, state) -> int:
        """Board-only key (blokus_wrapper.py:208-218): the engine's 64-bit board hash."""
        return int(np.asarray(state, dtype=np.uint8)[4 * W_HASH: 4 * W_HASH + 8].view(np.uint64)[0])

    @staticmethod
    def to_move(state) -> int:
        return int(np.asarray(state, dtype=np.uint8).view(np.int32)[W_TO_MOVE])

    def board_contents(self, state) -> np.ndarray:
        """[N, N] int8: 0 empty, k+1 colour k (the reference board's board_contents)."""
        occ = np.asarray(state, dtype=np.uint8)[:320].view(np.uint32).reshape(4, 20)[:, : self.board_size]
        cols = np.arange(self.board_size, dtype=np.uint32)
        out = np.zeros((self.board_size, self.board_size), dtype=np.int8)
        for k in range(self.number_of_players):
            out[((occ[k][:, None] >> cols) & 1).astype(bool)] = k + 1
        return out

    def display(self, state) -> None:
        print(self.board_contents(state))

    def get_sample_move(self, state):
        """blokus_wrapper.py:233-246: a uniformly random legal id (np.random)."""
        ids = np.nonzero(self.get_valid_moves(state, -1))[0]
        return int(np.random.choice(ids))

    def render(self, state, cell: int = 16) -> np.ndarray:
        """RGB image of the board (rows drawn bottom-up like blokus_wrapper.py:248-279)."""
        b = self.board_contents(state)[::-1]
        img = np.zeros((b.shape[0] * cell, b.shape[1] * cell, 3), dtype=np.uint8)
        for v, rgb in COLOURS.items():
            img[np.kron(b == v, np.ones((cell, cell), dtype=bool))] = rgb
        img[::cell, :, :] = 0
        img[:, ::cell, :] = 0
        return img
