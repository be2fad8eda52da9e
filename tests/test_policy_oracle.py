"""The CPU restatement of k_vec_policy (oracle/vecenv_oracle.py policy_sample) against the
reference's own ops, on the host: its exp / log polynomials within 3 ulp of libm; its draw's law
(chi-square vs softmax over the legal ids) and log-probs vs torch's
Categorical(logits=FilterLegalMoves(x)).log_prob (ppo/agent.py:27-42, 148-156) within f32
rounding; the filter's edge cases (a legal logit of exactly 0 masked under zero_masked; no
candidate -> every id uniform with log-prob 0, as torch gives the all -1e9 row)."""
import numpy as np
import torch
from scipy import stats

from oracle.vecenv_oracle import bk_expf, bk_logf, policy_sample, scan16_f32


def _mask_of(ids, W=15):
    m = np.zeros(W, dtype=np.uint64)
    for i in ids:
        m[i // 64] |= np.uint64(1) << np.uint64(i % 64)
    return m


def _reference_filter(x, legal):
    """FilterLegalMoves (ppo/agent.py:33-42) as written: x * mask, every 0 -> -1e9."""
    mask = torch.zeros_like(x)
    mask[:, legal] = 1
    out = x * mask
    out[out == 0] = -1e9
    return out


def test_exp_log_accuracy():
    x = -np.linspace(0, 79.9, 100001).astype(np.float32)
    ref = np.exp(x.astype(np.float64))
    assert np.max(np.abs(bk_expf(x) - ref) / ref) < 3 * 2.0 ** -23
    assert bk_expf(np.float32(0)) == 1.0 and bk_expf(np.float32(-81)) == 0.0
    y = np.linspace(1, 5000, 100001).astype(np.float32)
    assert np.max(np.abs(bk_logf(y) - np.log(y.astype(np.float64))) / np.maximum(np.log(y), 1e-3)) < 1e-6
    s = np.random.default_rng(0).random((4, 16)).astype(np.float32)
    np.testing.assert_allclose(scan16_f32(s), np.cumsum(s, axis=1), rtol=1e-6)


def test_policy_sample_law_and_logprob():
    rng = np.random.default_rng(1)
    E, A = 20000, 919
    row = (rng.standard_normal(A) * 2).astype(np.float32)
    legal = np.sort(rng.choice(A, 60, replace=False))
    row[legal[::6]] = 0.0  # legal ids at exactly 0: masked under zero_masked
    act, lp, new = policy_sample(np.tile(row, (E, 1)), np.tile(_mask_of(legal), (E, 1)), list(range(E)), True)
    assert len(new) == E and new[0] == 0x9E3779B97F4A7C15
    filt = _reference_filter(torch.from_numpy(row)[None], torch.from_numpy(legal))
    dist = torch.distributions.Categorical(logits=filt[0])
    np.testing.assert_allclose(lp, dist.log_prob(torch.from_numpy(act).long()).numpy(), rtol=2e-6, atol=2e-6)
    p = dist.probs.double().numpy()
    counts = np.bincount(act, minlength=A)
    assert counts[p == 0].sum() == 0
    keep = p > 0
    chi = (((counts[keep] - E * p[keep]) ** 2) / (E * p[keep])).sum()
    assert stats.chi2.sf(chi, keep.sum() - 1) > 1e-4
    act2, _, _ = policy_sample(np.tile(row, (E, 1)), np.tile(_mask_of(legal), (E, 1)), list(range(E)), False)
    assert np.isin(act2, legal[::6]).any()


def test_no_candidate_row_is_uniform_over_every_id():
    E, A = 30000, 919
    x = np.zeros((E, A), dtype=np.float32)
    legal = np.array([3, 70, 900])
    act, lp, _ = policy_sample(x, np.tile(_mask_of(legal), (E, 1)), list(range(E)), True)
    filt = _reference_filter(torch.from_numpy(x[:1]), torch.from_numpy(legal))
    want = torch.distributions.Categorical(logits=filt[0]).log_prob(torch.tensor([5]))
    assert float(want) == 0.0 and (lp == 0.0).all()
    counts = np.bincount(act, minlength=A)
    assert counts.shape[0] == A and stats.chisquare(counts).pvalue > 1e-4
