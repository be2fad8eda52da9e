"""Drop-in `MCTS` (blokus_rl/alphazero/mcts.py:7-99) on the GPU search engine.

`MCTS(game, nn)`, `.simulate(s, current_player, cpuct=1, epsilon_fix=True) -> scores` and
`.get_distribution(s, temperature) -> object array (K, 2) of [array([id]), prob]` behave as the
reference's (same selection rule, backup, tie-breaking, float64 statistics): the tree is a
one-tree BatchedMCTS. `nn` may be this package's BlokusNNetWrapper (device path: log-probs over
all ids, masked softmax inside k_expand_backup) or any object with the reference's
`predict(obs, mask) -> (p over legal ids, v)` (its p is handed to the engine as is).
"""
from __future__ import annotations

import numpy as np
import torch

from .batched_mcts import BatchedMCTS


# simulations per move assumed when the game carries no hparams.num_mcts_sims: the reference docs'
# arena setting (docs/README.md:159)
DEFAULT_SIMS = 200


def node_cap_for(game, sims: int | None = None) -> int:
    """Nodes one tree needs for a whole game: the reference tree grows without bound (mcts.py:67-70),
    a simulation adds at most one node and a game lasts at most pieces x players plies, so
    sims x max plies + 1 (sims from the game's hparams.num_mcts_sims / arena_num_mcts_sims, the
    largest of the two and DEFAULT_SIMS); a fuller tree raises EngineError at the expansion that
    does not fit (MCTS.simulate checks every expansion)."""
    eng = game.engine
    if sims is None:
        h = getattr(game, "hparams", None)
        cand = [int(getattr(h, k)) for k in ("num_mcts_sims", "arena_num_mcts_sims")
                if h is not None and isinstance(getattr(h, k, None), (int, float))]
        sims = max(cand + [DEFAULT_SIMS])
    return int(sims) * eng.num_pieces * eng.P + 1


class MCTS:
    def __init__(self, game, nn, node_cap: int | None = None, child_cap: int | None = None):
        self.game = game
        self.nn = nn
        eng = game.engine
        self._eng = eng
        if node_cap is None:
            node_cap = node_cap_for(game)
        self._m = BatchedMCTS(eng, 1, node_cap=node_cap, child_cap=child_cap or node_cap * (256 if eng.N >= 14 else 64))
        self._logp = torch.zeros((1, eng.A), dtype=torch.float32, device=eng.device)
        self._vals = torch.zeros((1, eng.P), dtype=torch.float32, device=eng.device)

    @property
    def tree(self):
        """Size view of the transposition table (the reference exposes its dict)."""
        return {"nodes": self._m.counters()["nodes"]}

    def simulate(self, s, current_player: int, cpuct: float = 1, epsilon_fix: bool = True):
        # epsilon_fix: sqrt(N.sum() + 1e-6) at the root, else sqrt(N.sum() + 0) (mcts.py:43); deeper
        # levels always take 1e-6 (the recursive call of mcts.py:50 passes the default)
        roots = self.game._dev(s)
        status, obs, mask = self._m.select(roots, None, float(cpuct), 1e-6 if epsilon_fix else 0.0)
        st = int(status[0])
        if st == 2:
            leaves, _ = self._m.leaf_info()
            _, scores = self._eng.game_ended(leaves)
            self._m.expand_backup(self._logp, self._vals, prior_mode=1)
            self._m.check()
            return scores[0].cpu().numpy()
        if st != 1:
            self._m.check()
            raise RuntimeError("MCTS select failed")
        if hasattr(self.nn, "predict_batch"):
            logp, v = self.nn.predict_batch(obs)
            self._m.expand_backup(logp, v, prior_mode=0)
            self._m.check()  # a full node/child table raises here instead of distorting pi
            return v[0].cpu().numpy()
        mask_f = self._eng.unpack_mask(mask)[0].cpu().numpy().astype(np.float64)
        p, v = self.nn.predict(obs[0].cpu().numpy(), mask_f)
        ids = torch.from_numpy(np.nonzero(mask_f)[0]).to(self._eng.device)
        self._logp.zero_()
        self._logp[0, ids] = torch.as_tensor(np.atleast_1d(p), dtype=torch.float32, device=self._eng.device)
        self._vals[0] = torch.as_tensor(np.asarray(v, dtype=np.float32), device=self._eng.device)
        self._m.expand_backup(self._logp, self._vals, prior_mode=1)
        self._m.check()
        return v

    def get_distribution(self, s, temperature):
        roots = self.game._dev(s)
        ids, pi, counts = self._m.root_policy(roots, None, float(temperature))
        K = int(counts[0])
        if K < 0:
            raise KeyError(self.game.string_representation(s))
        out = np.zeros((K, 2), dtype=np.object_)
        out[:, 0] = [np.array([i]) for i in ids[0, :K].cpu().tolist()]
        out[:, 1] = pi[0, :K].cpu().numpy()
        return out
