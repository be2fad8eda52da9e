"""TEST INFRASTRUCTURE ONLY — Python face of the CPU oracle.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It is the checker the HIP product is compared against, never a fallback for it.

* `Oracle`: ctypes binding of oracle/blokus_oracle.c (the C restatement of the colosseumrl
  rules pinned by the reference's recordings; see that file's header).
* `mcts_*`: a pure-Python restatement of the reference search, `MCTS.simulate` /
  `MCTS.get_distribution` (blokus_rl/alphazero/mcts.py:13-99), in float64 arithmetic — the
  arithmetic the reference gets under its pinned numpy==1.25.2 (setup.py) where every
  np.float32 scalar meeting a Python number promotes to float64.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libblokus_oracle.so")
STATE_BYTES = 384

_c_u8p = ctypes.POINTER(ctypes.c_uint8)


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def _load():
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    lib.bko_create.restype = ctypes.c_void_p
    lib.bko_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.bko_destroy.argtypes = [ctypes.c_void_p]
    for name in ("bko_action_size", "bko_num_pieces"):
        getattr(lib, name).argtypes = [ctypes.c_void_p]
        getattr(lib, name).restype = ctypes.c_int
    lib.bko_action_table.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.bko_action_cells.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.bko_init_state.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.bko_legal_mask.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lib.bko_legal_mask.restype = ctypes.c_int
    lib.bko_legal_mask_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_void_p]
    lib.bko_next_state.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lib.bko_next_state.restype = ctypes.c_int
    lib.bko_game_ended.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.bko_game_ended.restype = ctypes.c_int
    lib.bko_square_counts.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.bko_observe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.bko_hash.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.bko_hash.restype = ctypes.c_uint64
    lib.bko_make_state.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p]
    return lib


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _load()
    return _LIB


def _ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


class Oracle:
    """CPU restatement of the rules for one preset (board N, players P, max piece cells)."""

    def __init__(self, board_size: int = 20, num_players: int = 4, max_piece_cells: int = 5):
        self.L = lib()
        self.N, self.P, self.maxc = board_size, num_players, max_piece_cells
        self.h = self.L.bko_create(board_size, num_players, max_piece_cells)
        if not self.h:
            raise ValueError("bad preset")
        self.A = self.L.bko_action_size(self.h)
        self.W = (self.A + 63) // 64
        self.num_pieces = self.L.bko_num_pieces(self.h)

    def __del__(self):
        try:
            self.L.bko_destroy(self.h)
        except Exception:  # pragma: no cover
            pass

    # tables --------------------------------------------------------------------------------
    def action_table(self) -> np.ndarray:
        out = np.zeros((self.A, 4), dtype=np.int32)
        self.L.bko_action_table(self.h, _ptr(out))
        return out

    def action_cells(self) -> np.ndarray:
        out = np.zeros((self.A, 5), dtype=np.int16)
        self.L.bko_action_cells(self.h, _ptr(out))
        return out

    # states --------------------------------------------------------------------------------
    def init_state(self) -> np.ndarray:
        st = np.zeros(STATE_BYTES, dtype=np.uint8)
        self.L.bko_init_state(self.h, _ptr(st))
        return st

    def legal_mask(self, st: np.ndarray, player: int = -1):
        mask = np.zeros(self.W, dtype=np.uint64)
        n = self.L.bko_legal_mask(self.h, _ptr(st), player, _ptr(mask))
        return mask, n

    def legal_ids(self, st: np.ndarray, player: int = -1) -> np.ndarray:
        mask, _ = self.legal_mask(st, player)
        bits = np.unpackbits(mask.view(np.uint8), bitorder="little")[: self.A]
        return np.nonzero(bits)[0]

    def legal_mask_batch(self, states: np.ndarray):
        states = np.ascontiguousarray(states, dtype=np.uint8)
        B = states.shape[0]
        masks = np.zeros((B, self.W), dtype=np.uint64)
        counts = np.zeros(B, dtype=np.int32)
        self.L.bko_legal_mask_batch(self.h, _ptr(states), B, _ptr(masks), _ptr(counts))
        return masks, counts

    def next_state(self, st: np.ndarray, action: int):
        out = np.zeros(STATE_BYTES, dtype=np.uint8)
        nxt = self.L.bko_next_state(self.h, _ptr(st), int(action), _ptr(out))
        if nxt < 0:
            raise KeyError(f"illegal action {action}")
        return out, nxt

    def game_ended(self, st: np.ndarray):
        scores = np.zeros(self.P, dtype=np.float64)
        ended = self.L.bko_game_ended(self.h, _ptr(st), _ptr(scores))
        return scores if ended else None

    def square_counts(self, st: np.ndarray) -> np.ndarray:
        out = np.zeros(self.P, dtype=np.int32)
        self.L.bko_square_counts(self.h, _ptr(st), _ptr(out))
        return out

    def observe(self, st: np.ndarray) -> np.ndarray:
        obs = np.zeros((2 * self.P, self.N, self.N), dtype=np.float32)
        self.L.bko_observe(self.h, _ptr(st), _ptr(obs))
        return obs

    def hash(self, st: np.ndarray) -> int:
        return int(self.L.bko_hash(self.h, _ptr(st)))

    def make_state(self, cells: np.ndarray, pieces, to_move: int, ply: int = 0, flags: int = 0):
        cells = np.ascontiguousarray(cells, dtype=np.int8)
        pieces = np.ascontiguousarray(np.asarray(pieces, dtype=np.uint32).reshape(4))
        st = np.zeros(STATE_BYTES, dtype=np.uint8)
        self.L.bko_make_state(self.h, _ptr(cells), _ptr(pieces), to_move, ply, flags, _ptr(st))
        return st

    @staticmethod
    def to_move(st: np.ndarray) -> int:
        return int(st[344:348].view(np.int32)[0])

    # random playouts (SURVEY.md §8d config 2 recipe) --------------------------------------
    def random_board(self, seed: int, max_plies: int = 60) -> np.ndarray:
        """default_rng(seed): t ~ U{0..max_plies}, then t uniform-random legal plies."""
        rng = np.random.default_rng(seed)
        t = int(rng.integers(0, max_plies + 1))
        st = self.init_state()
        for _ in range(t):
            if self.game_ended(st) is not None:
                break
            ids = self.legal_ids(st)
            st, _ = self.next_state(st, int(ids[int(rng.integers(len(ids)))]))
        return st


# --------------------------------------------------------------------------- MCTS oracle
class MCTSOracle:
    """Pure-Python restatement of the reference MCTS (blokus_rl/alphazero/mcts.py:7-99).

    `evaluate(state, player) -> (ids, p[K], v[P])` supplies the leaf evaluation the reference
    gets from `nn.predict(obs, mask)` (mcts.py:65-66); tests feed identical p/v to the GPU
    engine. Arithmetic is float64 throughout (see module docstring)."""

    def __init__(self, oracle: Oracle, evaluate):
        self.o = oracle
        self.evaluate = evaluate
        self.tree: dict[int, dict] = {}
        self.terminal_hits = 0

    def simulate(self, s: np.ndarray, cpuct: float = 1.0, epsilon_fix: bool = True):
        h = self.o.hash(s)
        player = Oracle.to_move(s)
        if h in self.tree:  # mcts.py:39-57
            node = self.tree[h]
            N, Q, P = node["N"], node["Q"], node["P"]
            sq = math.sqrt(float(sum(N)) + (1e-6 if epsilon_fix else 0))  # mcts.py:43
            best, best_i = -math.inf, 0
            for i in range(len(N)):
                u = cpuct * P[i] * sq / (1 + N[i])
                hv = Q[i] + u
                if hv > best:
                    best, best_i = hv, i
            s2, p2 = self.o.next_state(s, node["ids"][best_i])
            scores = self.simulate(s2)  # cpuct, epsilon_fix not forwarded (mcts.py:50)
            v = float(scores[p2])
            n, q = N[best_i], Q[best_i]
            Q[best_i] = (n * q + v) / (n + 1)
            N[best_i] += 1
            return scores
        ended = self.o.game_ended(s)  # mcts.py:59-61
        if ended is not None:
            self.terminal_hits += 1
            return ended
        ids, p, v = self.evaluate(s, player)
        self.tree[h] = {
            "ids": [int(i) for i in ids],
            "N": [0] * len(ids),
            "Q": [0.0] * len(ids),
            "P": [float(x) for x in np.asarray(p, dtype=np.float32).reshape(-1)],
        }
        return np.asarray(v, dtype=np.float64)

    def get_distribution(self, s: np.ndarray, temperature: float):
        """mcts.py:73-99: N^(1/T) normalised; T=0 -> one-hot argmax; all-zero -> uniform."""
        node = self.tree[self.o.hash(s)]
        N = np.array(node["N"], dtype=np.float64)
        if temperature == 0:
            raised = np.zeros_like(N)
            raised[int(np.argmax(N))] = 1
        else:
            raised = np.power(N, 1.0 / temperature)
        total = raised.sum()
        if total == 0:
            raised[:] = 1
            total = raised.sum()
        return np.array(node["ids"]), raised / total
