"""TEST INFRASTRUCTURE ONLY — CPU restatement of the config-5 vector env (one env at a time),
the same rules (oracle/blokus_oracle.c) and the same per-env random stream as
blokus_rl_amd/csrc/vecenv.hip, so the two compare bit for bit. The env restates blokus_gym
`blokus-simple-v0` as the reference PPO uses it (ppo/trainer.py:128-175; docs/README.md:47-51).

`policy_sample` restates policy_draw16 (the rollout's masked-policy draw of k_vec_policy and of
the fused k_vec_step7, ppo/agent.py:27-42 + :148-156, ppo/trainer.py:144-155) in numpy float32 with
the kernel's exact operation order: its exp / log polynomials, the per-lane sums, the 16-lane scan
and the inverse-CDF walk, so actions and log-probs compare bit for bit."""
from __future__ import annotations

import numpy as np

from .oracle import Oracle

M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
F32 = np.float32


def mix64(x: int) -> int:
    """splitmix64 finalizer of x + golden (common.h mix64)."""
    z = (x + GOLDEN) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def bk_expf(x):
    """vecenv.hip bk_expf: x <= 0 in float32; 0 below -80."""
    x = np.asarray(x, dtype=F32)
    ok = x >= F32(-80.0)
    xc = np.where(ok, x, F32(0))
    n = np.rint(xc * F32(1.44269502))
    r = (xc - n * F32(0.693145752)) - n * F32(1.42860677e-6)
    p = np.full_like(r, F32(1.38888892e-3))
    for c in (8.33333377e-3, 4.16666679e-2, 0.166666672, 0.5, 1.0, 1.0):
        p = p * r + F32(c)
    pw = ((n.astype(np.int32) + 127) << 23).astype(np.int32).view(F32)
    return np.where(ok, p * pw, F32(0)).astype(F32)


def bk_logf(x):
    """vecenv.hip bk_logf: x >= 1 finite, float32."""
    x = np.ascontiguousarray(np.asarray(x, dtype=F32))
    bits = x.view(np.int32)
    e = ((bits >> 23) & 255) - 127
    f = ((bits & 0x7FFFFF) | 0x3F800000).astype(np.int32).view(F32)
    big = f > F32(1.41421354)
    f = np.where(big, f * F32(0.5), f).astype(F32)
    e = np.where(big, e + 1, e)
    s = (f - F32(1)) / (f + F32(1))
    s2 = s * s
    q = np.full_like(s, F32(0.111111112))
    for c in (0.142857149, 0.200000003, 0.333333343, 1.0):
        q = q * s2 + F32(c)
    return (e.astype(F32) * F32(0.693147182) + (F32(2) * s) * q).astype(F32)


def scan16_f32(s):
    """The 16-lane Hillis-Steele scan of policy_draw16 (DPP row_shr 1, 2, 4, 8) over s [..., 16]."""
    x = np.array(s, dtype=F32)
    lane = np.arange(16)
    for d in (1, 2, 4, 8):
        src = x.copy()
        sel = lane >= d
        x[..., sel] = src[..., lane[sel] - d] + src[..., sel]
    return x


def policy_sample(logits, masks, rng, zero_masked: bool = True):
    """policy_draw16 (vecenv.hip; k_vec_policy and the fused k_vec_step7 draw) on the CPU.
    logits [E, A] f32, masks [E, W] u64 (the agent's legal ids), rng: E int states.
    -> (actions int32 [E], logp f32 [E], new rng states). Lane j of an env owns mask words j, j + 16,
    ...; its candidates in ascending id order."""
    logits = np.asarray(logits, dtype=F32)
    masks = np.asarray(masks, dtype=np.uint64)
    E, A = logits.shape
    ids = np.arange(A)
    lane_of = (ids // 64) % 16
    bits = ((masks[:, ids // 64] >> (ids % 64).astype(np.uint64)) & np.uint64(1)).astype(bool)
    cand = bits & ((logits != 0) if zero_masked else True)
    none = ~cand.any(axis=1)
    X = logits.copy()
    X[none] = F32(-1e9)
    cand[none] = True
    m = np.where(cand, X, F32(-np.inf)).max(axis=1).astype(F32)
    P = np.where(cand, bk_expf(np.where(cand, X - m[:, None], F32(0))), F32(0)).astype(F32)
    s = np.zeros((E, 16), dtype=F32)
    for a in range(A):  # each lane's sum in ascending id order
        j = lane_of[a]
        s[:, j] = np.where(cand[:, a], s[:, j] + P[:, a], s[:, j])
    incl = scan16_f32(s)
    S = incl[:, 15].copy()
    z = [mix64(int(st)) for st in rng]
    new_rng = [(int(st) + GOLDEN) & M64 for st in rng]
    u = np.array([zz >> 40 for zz in z], dtype=np.uint32).astype(F32) * F32(2.0 ** -24)
    target = (S * u).astype(F32)
    over = incl > target[:, None]
    pos = s > F32(0)
    last_pos = np.where(pos.any(1), 15 - pos[:, ::-1].argmax(1), 0)
    sel = np.where(over.any(1), over.argmax(1), last_pos)
    er = np.arange(E)
    acc = np.where(sel > 0, incl[er, np.maximum(sel - 1, 0)], F32(0)).astype(F32)
    pick = np.full(E, -1)
    last = np.full(E, -1)
    for a in range(A):  # the selected lane's walk, ids ascending
        live = (lane_of[a] == sel) & cand[:, a] & (pick < 0)
        pa = P[:, a]
        ok = live & (pa > F32(0))
        acc = np.where(ok, acc + pa, acc).astype(F32)
        last = np.where(ok, a, last)
        pick = np.where(ok & (acc > target), a, pick)
    pick = np.where(pick < 0, last, pick)
    good = pick >= 0
    pk = np.maximum(pick, 0)
    actions = np.where(good, pk, A).astype(np.int32)
    logp = np.where(good, X[er, pk] - (m + bk_logf(np.maximum(S, F32(1)))), F32(np.nan)).astype(F32)
    return actions, logp, new_rng


def rng_index(state: int, K: int):
    state = (state + GOLDEN) & M64
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

    def sample_policy(self, logits, zero_masked: bool = True):
        """The agent's moves from its policy logits [E, A] over each env's current legal mask
        (k_vec_policy); advances each env's stream by one draw. -> (actions, logp)."""
        masks = np.stack([self.mask(e) for e in range(self.E)])
        act, logp, self.rng = policy_sample(logits, masks, self.rng, zero_masked)
        return act, logp

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
