"""CPU restatement of the PPO trainer's array math (TEST INFRASTRUCTURE ONLY — imported by tests/,
never by the product path). Pinned against tests/golden/ppo_golden.npz, which holds outputs of
the reference's own code (tests/golden/make_ppo_golden.py).

* gae_f32 — PPOTrainer._compute_gae (blokus_rl/ppo/trainer.py:177-211) in numpy float32 with the
  reference's operation order: delta = (r + (g*nv)*nnt) - v; adv = delta + (f32(g*lam)*nnt)*last.
* filter_legal — FilterLegalMoves (blokus_rl/ppo/agent.py:27-42): x*mask, zeros -> -1e9.
"""
import numpy as np


def gae_f32(rewards, values, dones, next_value, next_done, gamma, gae_lambda):
    r = np.asarray(rewards, np.float32)
    v = np.asarray(values, np.float32)
    d = np.asarray(dones, np.float32)
    T = r.shape[0]
    g = np.float32(gamma)
    gl = np.float32(gamma * gae_lambda)  # Python double product, rounded once (trainer.py:206-209)
    one = np.float32(1.0)
    adv = np.zeros_like(r)
    last = np.zeros(r.shape[1], np.float32)
    for t in range(T - 1, -1, -1):
        if t == T - 1:
            nnt = one - np.asarray(next_done, np.float32).reshape(-1)
            nv = np.asarray(next_value, np.float32).reshape(-1)
        else:
            nnt = one - d[t + 1]
            nv = v[t + 1]
        delta = (r[t] + (g * nv) * nnt) - v[t]
        last = delta + (gl * nnt) * last
        adv[t] = last
    return adv, adv + v


def filter_legal(x, mask):
    out = np.asarray(x, np.float32) * np.asarray(mask, np.float32)
    out[out == 0] = np.float32(-1e9)
    return out
