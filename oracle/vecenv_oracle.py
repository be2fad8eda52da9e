"""TEST INFRASTRUCTURE ONLY — CPU restatement of the config-5 vector env (one env at a time),
the same rules (oracle/blokus_oracle.c) and the same per-env random stream as
blokus_rl_amd/csrc/vecenv.hip, so the two compare bit for bit. The env restates blokus_gym
`blokus-simple-v0` as the reference PPO uses it (ppo/trainer.py:128-175; docs/README.md:47-51)."""
from __future__ import annotations

import numpy as np

from .oracle import Oracle

M64 = (1 << 64) - 1


def rng_index(state: int, K: int):
    state = (state + 0x9E3779B97F4A7C15) & M64
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    z ^= z >> 31
    return state, ((z >> 32) * K) >> 32


class VecEnvOracle:
    def __init__(self, E: int, board_size: int = 7, max_piece_cells: int = 4):
        self.o = Oracle(board_size, 2, max_piece_cells)
        self.E = E
        self.states = [self.o.init_state() for _ in range(E)]
        self.rng = [0] * E

    def reset(self, seed: int = 0):
        self.states = [self.o.init_state() for _ in range(self.E)]
        self.rng = [(seed * 1_000_003 + e) & M64 for e in range(self.E)]

    def obs(self, e):
        occ = self.states[e][:320].view(np.uint32).reshape(4, 20)
        N = self.o.N
        out = np.zeros((N, N), dtype=np.uint8)
        for r in range(N):
            for c in range(N):
                out[r, c] = 1 if (occ[0, r] >> c) & 1 else (2 if (occ[1, r] >> c) & 1 else 0)
        return out

    def mask(self, e):
        return self.o.legal_mask(self.states[e], 0)[0]

    def step(self, e: int, action: int):
        s = self.states[e]
        if action < 0:
            ids = self.o.legal_ids(s, 0)
            self.rng[e], k = rng_index(self.rng[e], len(ids))
            action = int(ids[k])
        try:
            s, _ = self.o.next_state(s, action)
        except KeyError:
            self.states[e] = self.o.init_state()
            return -1.0, 1
        while self.o.game_ended(s) is None and Oracle.to_move(s) == 1:
            ids = self.o.legal_ids(s, 1)
            self.rng[e], k = rng_index(self.rng[e], len(ids))
            s, _ = self.o.next_state(s, int(ids[k]))
        if self.o.game_ended(s) is not None:
            sq = self.o.square_counts(s)
            rew = 1.0 if sq[0] > sq[1] else (-1.0 if sq[0] < sq[1] else 0.0)
            self.states[e] = self.o.init_state()
            return rew, 1
        self.states[e] = s
        return 0.0, 0
