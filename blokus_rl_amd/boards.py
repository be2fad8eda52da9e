"""Synthetic board batches for the legal-move benchmark.

Board b: `numpy.random.default_rng(seed0 + b)` draws t ~ U{0..max_plies}, then plays t uniform
random legal placements (stopping at a terminal board). Every placement is computed by the HIP
engine (legal ids + next state); the host only draws the random indices, so the same recipe on
the oracle (oracle.Oracle.random_board) reproduces the boards byte for byte.
"""
from __future__ import annotations

import numpy as np
import torch

from .engine import Engine


def random_boards(eng: Engine, B: int, seed0: int = 0, max_plies: int = 60, cap: int = 4096) -> torch.Tensor:
    rngs = [np.random.default_rng(seed0 + b) for b in range(B)]
    target = np.array([int(r.integers(0, max_plies + 1)) for r in rngs], dtype=np.int64)
    states = eng.init_states(B)
    for ply in range(int(target.max(initial=0))):
        ended, _ = eng.game_ended(states)
        ids, counts = eng.legal_ids(states, cap=cap)
        ended_h = ended.cpu().numpy()
        counts_h = counts.cpu().numpy()
        if (counts_h < 0).any():
            raise RuntimeError("legal-id capacity exceeded")
        pick = np.full(B, -1, dtype=np.int64)
        for b in range(B):
            if ply < target[b] and not ended_h[b]:
                pick[b] = int(rngs[b].integers(counts_h[b]))
        sel = torch.from_numpy(pick).to(eng.device)
        act = torch.where(sel >= 0, ids.gather(1, sel.clamp(min=0).view(-1, 1)).view(-1),
                          torch.full_like(sel, -1, dtype=torch.int32).to(torch.int32))
        act = act.to(torch.int32).contiguous()
        states, _, status = eng.next_state(states, act)
        if int(status.max().item()) != 0:
            raise RuntimeError("engine rejected a legal id")
    return states
