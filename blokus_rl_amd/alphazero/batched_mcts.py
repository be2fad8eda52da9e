"""Batched MCTS: T trees on one GPU, one simulation in flight per tree (bk_mcts_* C-ABI).

A simulation of the reference `MCTS.simulate` (blokus_rl/alphazero/mcts.py:13-71) is
`select()` -> one batched net forward over every tree's leaf -> `expand_backup()`. Because each
tree keeps exactly one simulation in flight, each tree's sequence of visits is the one the
reference's sequential recursion produces for the same priors and values.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ..engine import Engine, EngineError, _check, _ptr


class BatchedMCTS:
    def __init__(self, eng: Engine, trees: int, node_cap: int = 8192, child_cap: int | None = None):
        self.eng = eng
        self.lib = eng.lib
        self.T = trees
        self.node_cap = node_cap
        if child_cap is None:
            # ~ node_cap nodes x mean branching; 20x20 trajectories average K ~ 211
            per_node = 256 if eng.N >= 14 else 64
            child_cap = trees * node_cap * per_node
        self.child_cap = child_cap
        h = ctypes.c_void_p()
        with torch.cuda.device(eng.device):
            _check(self.lib.bk_mcts_create(eng.h, trees, node_cap, ctypes.c_int64(child_cap), ctypes.byref(h)))
        self.h = h
        dev = eng.device
        self.status = torch.zeros(trees, dtype=torch.int32, device=dev)
        self.obs = torch.zeros((trees,) + eng.obs_shape, dtype=torch.float32, device=dev)
        self.leaf_mask = torch.zeros((trees, eng.W), dtype=torch.int64, device=dev)

    def __del__(self):
        try:
            if getattr(self, "h", None):
                self.lib.bk_mcts_destroy(self.h)
                self.h = None
        except Exception:  # pragma: no cover
            pass

    def _s(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.eng.device).cuda_stream)

    def reset(self, flags: torch.Tensor | None = None):
        _check(self.lib.bk_mcts_reset(self.h, _ptr(flags), self._s()))

    def select(self, roots: torch.Tensor, active: torch.Tensor | None, cpuct: float = 1.0, root_eps: float = 1e-6):
        """Descend every active tree to a leaf; returns (status[T], obs[T,2P,N,N], mask[T,W]).
        root_eps: the root's term under the square root of mcts.py:43 (1e-6 = epsilon_fix, 0 = not)."""
        if root_eps == 1e-6:
            _check(self.lib.bk_mcts_select(self.h, _ptr(roots), _ptr(active), float(cpuct), _ptr(self.status),
                                           _ptr(self.obs), _ptr(self.leaf_mask), self._s()))
        else:
            _check(self.lib.bk_mcts_select_eps(self.h, _ptr(roots), _ptr(active), float(cpuct), float(root_eps),
                                               _ptr(self.status), _ptr(self.obs), _ptr(self.leaf_mask), self._s()))
        return self.status, self.obs, self.leaf_mask

    def expand_backup(self, logp: torch.Tensor | None, values: torch.Tensor, prior_mode: int = 0):
        """prior_mode 0: dense logits/log-probs [T, A]; 1: priors at the legal ids (test hook);
        2: the sparse logits of leaf_logits() (logp None)."""
        assert values.dtype == torch.float32 and values.shape == (self.T, self.eng.P)
        if prior_mode != 2:
            assert logp.dtype == torch.float32 and logp.shape == (self.T, self.eng.A)
        _check(self.lib.bk_mcts_expand_backup(self.h, _ptr(logp), _ptr(values), prior_mode, self._s()))

    def leaf_logits(self, feat: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor):
        """Policy logits of each leaf's legal ids only (bk_mcts_leaf_logits): feat [T, F] f32,
        weight [A, F], bias [A] — the policy head's last Linear — for expand_backup(mode 2)."""
        assert feat.dtype == torch.float32 and feat.shape[0] == self.T and feat.stride(1) == 1
        assert weight.is_contiguous() and weight.shape == (self.eng.A, feat.shape[1]) and bias.shape == (self.eng.A,)
        _check(self.lib.bk_mcts_leaf_logits(self.h, ctypes.c_void_p(feat.data_ptr()), feat.stride(0), feat.shape[1],
                                            _ptr(weight), _ptr(bias), self._s()))

    def leaf_step(self, feat: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, values: torch.Tensor,
                  roots: torch.Tensor | None = None, active: torch.Tensor | None = None, cpuct: float = 1.0,
                  want_mask: bool = True):
        """leaf_logits(feat, weight, bias) + expand_backup(None, values, 2) and, when roots is given,
        the next select(roots, active, cpuct) in one launch (bk_mcts_leaf_step; the same trees
        bitwise). Returns select's (status, obs, mask) or None. want_mask=False: the next leaves'
        bitmasks are not copied out (the engine keeps its own for the next step; self-play's
        captured graph reads only status and obs), and the returned mask is stale."""
        assert feat.dtype == torch.float32 and feat.shape[0] == self.T and feat.stride(1) == 1
        assert weight.is_contiguous() and weight.shape == (self.eng.A, feat.shape[1]) and bias.shape == (self.eng.A,)
        assert values.dtype == torch.float32 and values.shape == (self.T, self.eng.P)
        sel = roots is not None
        _check(self.lib.bk_mcts_leaf_step(self.h, ctypes.c_void_p(feat.data_ptr()), feat.stride(0), feat.shape[1],
                                          _ptr(weight), _ptr(bias), _ptr(values), int(sel), _ptr(roots),
                                          _ptr(active), float(cpuct), _ptr(self.status) if sel else None,
                                          _ptr(self.obs) if sel else None,
                                          _ptr(self.leaf_mask) if sel and want_mask else None,
                                          self._s()))
        return (self.status, self.obs, self.leaf_mask) if sel else None

    def root_policy(self, roots: torch.Tensor, active: torch.Tensor | None, temperature: float, cap: int = 2048,
                    zero: bool = True):
        """ids/pi rows of every root (k_root); zero=False leaves the entries past each row's count
        unwritten (bk_ply_policy reads only the first counts[t])."""
        alloc = torch.zeros if zero else torch.empty
        ids = alloc((self.T, cap), dtype=torch.int32, device=self.eng.device)
        pi = alloc((self.T, cap), dtype=torch.float64, device=self.eng.device)
        counts = alloc(self.T, dtype=torch.int32, device=self.eng.device)
        _check(self.lib.bk_mcts_root_policy(self.h, _ptr(roots), _ptr(active), float(temperature), _ptr(ids),
                                            _ptr(pi), cap, _ptr(counts), self._s()))
        return ids, pi, counts

    def root_stats(self, roots: torch.Tensor, active: torch.Tensor | None = None, cap: int = 2048):
        dev = self.eng.device
        ids = torch.zeros((self.T, cap), dtype=torch.int32, device=dev)
        n = torch.zeros((self.T, cap), dtype=torch.int32, device=dev)
        q = torch.zeros((self.T, cap), dtype=torch.float64, device=dev)
        p = torch.zeros((self.T, cap), dtype=torch.float32, device=dev)
        counts = torch.zeros(self.T, dtype=torch.int32, device=dev)
        _check(self.lib.bk_mcts_root_stats(self.h, _ptr(roots), _ptr(active), _ptr(ids), _ptr(n), _ptr(q), _ptr(p),
                                           cap, _ptr(counts), self._s()))
        return ids, n, q, p, counts

    def leaf_info(self):
        states = torch.empty((self.T, 384), dtype=torch.uint8, device=self.eng.device)
        depths = torch.empty(self.T, dtype=torch.int32, device=self.eng.device)
        _check(self.lib.bk_mcts_leaf_info(self.h, _ptr(states), _ptr(depths), self._s()))
        return states, depths

    def counters(self) -> dict:
        out = np.zeros(8, dtype=np.int64)
        _check(self.lib.bk_mcts_counters(self.h, out.ctypes.data_as(ctypes.c_void_p), self._s()))
        keys = ["nodes", "children", "levels", "expanded", "terminal", "errors", "scanned", "leaf_children"]
        return {k: int(out[i]) for i, k in enumerate(keys)}

    def check(self):
        c = self.counters()
        if c["errors"]:
            raise EngineError(f"MCTS capacity/consistency error flags {c['errors']:#x} (counters {c})")
        return c


def smoke_search(eng: Engine, oracle) -> None:
    """Tiny search on cuda:0 (used by __graft_entry__.smoke): 4 trees x 8 simulations with a
    uniform prior, checked for tree growth, visit accounting and legal root children."""
    T = 4
    m = BatchedMCTS(eng, T, node_cap=64, child_cap=T * 64 * 700)
    roots = eng.init_states(T)
    logp = torch.zeros((T, eng.A), dtype=torch.float32, device=eng.device)
    vals = torch.zeros((T, eng.P), dtype=torch.float32, device=eng.device)
    for _ in range(8):
        m.select(roots, None, 1.0)
        m.expand_backup(logp, vals)
    c = m.check()
    assert c["expanded"] == T * 8, c
    ids, n, q, p, counts = m.root_stats(roots)
    K = int(counts[0])
    ref_ids = oracle.legal_ids(roots[0].cpu().numpy())
    assert K == len(ref_ids) and (ids[0, :K].cpu().numpy() == ref_ids).all()
    assert int(n[0, :K].sum()) == 7  # first simulation expands the root
    assert abs(float(p[0, :K].sum()) - 1.0) < 1e-5
