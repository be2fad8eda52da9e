"""GPU batched MCTS against golden vectors from the reference's own mcts.py.

Trees of the same (preset, cpuct) run side by side in one BatchedMCTS (one simulation in flight
per tree). Priors/values come from the same deterministic stand-in net the golden generator fed
the reference (prior_mode 1 = the prior is handed over as is), so the comparison is bit-exact:
root child ids, N, Q (float64), P, every recorded node's visited children, get_distribution at
T=1 and T=0, across moves on the reused tree. A second test checks the product prior path
(prior_mode 0: masked log-softmax of the net output, neural_network.py:159-173) against torch
within float32 tolerance."""
from collections import defaultdict

import numpy as np
import pytest
import torch

from mcts_golden_util import load_cases, prior_value, state_of, unhex

pytestmark = pytest.mark.gpu

CASES = load_cases()


def _groups():
    g = defaultdict(list)
    for k, c in enumerate(CASES):
        g[(tuple(c["preset"]), c["cpuct"], c.get("epsilon_fix", True))].append(k)
    return sorted(g.items())


def _bits_to_ids(words: np.ndarray, A: int) -> np.ndarray:
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:A]
    return np.nonzero(bits)[0]


@pytest.fixture(scope="module")
def engines():
    from blokus_rl_amd.engine import Engine
    return {p: Engine(*p) for p in {tuple(c["preset"]) for c in CASES}}


@pytest.mark.parametrize("group", _groups(), ids=lambda g: f"{g[0][0]}-cpuct{g[0][1]}{'' if g[0][2] else '-noeps'}")
def test_batched_mcts_matches_reference(engines, group):
    from blokus_rl_amd.alphazero.batched_mcts import BatchedMCTS
    from oracle.oracle import Oracle

    (preset, cpuct, eps_fix), case_ids = group
    eng = engines[preset]
    o = Oracle(*preset)
    dev = eng.device
    T = len(case_ids)
    m = BatchedMCTS(eng, T, node_cap=4096, child_cap=T * 4096 * (700 if preset[0] == 20 else 200))
    cases = [CASES[k] for k in case_ids]
    rounds = max(len(c["moves"]) for c in cases)
    logp = torch.zeros((T, eng.A), dtype=torch.float32, device=dev)
    vals = torch.zeros((T, eng.P), dtype=torch.float32, device=dev)
    for r in range(rounds):
        act_round = [r < len(c["moves"]) for c in cases]
        roots_h = np.stack([state_of(c["moves"][r]["root"]) if a else state_of(c["moves"][0]["root"])
                            for c, a in zip(cases, act_round)])
        roots = torch.from_numpy(roots_h).to(dev)
        sims = [c["moves"][r]["sims"] if a else 0 for c, a in zip(cases, act_round)]
        for sim in range(max(sims)):
            active = torch.tensor([1 if sim < s else 0 for s in sims], dtype=torch.int32, device=dev)
            status, _, mask = m.select(roots, active, float(cpuct), 1e-6 if eps_fix else 0.0)
            st_h = status.cpu().numpy()
            leaves, _ = m.leaf_info()
            leaves_h = leaves.cpu().numpy()
            mask_h = mask.cpu().numpy().view(np.uint64)
            logp.zero_()
            vals.zero_()
            for t in range(T):
                if st_h[t] == 1:
                    ids = _bits_to_ids(mask_h[t], eng.A)
                    assert (ids == o.legal_ids(leaves_h[t])).all()
                    p, v = prior_value(o.hash(leaves_h[t]), len(ids), eng.P)
                    logp[t, torch.from_numpy(ids).to(dev)] = torch.from_numpy(p).to(dev)
                    vals[t] = torch.from_numpy(v).to(dev)
            m.expand_backup(logp, vals, prior_mode=1)
        m.check()
        active = torch.tensor([1 if a else 0 for a in act_round], dtype=torch.int32, device=dev)
        ids, n, q, p, counts = m.root_stats(roots, active)
        pid, pi1, pc = m.root_policy(roots, active, 1.0)
        _, pi0, _ = m.root_policy(roots, active, 0.0)
        for t, c in enumerate(cases):
            if not act_round[t]:
                continue
            mv = c["moves"][r]
            K = int(counts[t])
            assert K == len(mv["ids"])
            assert ids[t, :K].cpu().tolist() == mv["ids"]
            assert p[t, :K].double().cpu().tolist() == unhex(mv["P"])
            assert pi1[t, :K].cpu().tolist() == unhex(mv["dist_T1"])
            assert pi0[t, :K].cpu().tolist() == unhex(mv["dist_T0"])
            assert pid[t, :K].cpu().tolist() == mv["ids"]
            # every recorded node of the reference tree, visited children bit-exact
            for rec in mv["nodes"]:
                node_roots = roots.clone()
                node_roots[t] = torch.from_numpy(state_of(rec["state"])).to(dev)
                only = torch.zeros(T, dtype=torch.int32, device=dev)
                only[t] = 1
                _, nn_, qq, _, cc = m.root_stats(node_roots, only)
                Kn = int(cc[t])
                assert Kn == rec["K"]
                nh, qh = nn_[t, :Kn].cpu().numpy(), qq[t, :Kn].cpu().numpy()
                got = [[i, int(nh[i]), float(qh[i])] for i in range(Kn) if nh[i] > 0]
                assert got == [[i, nv, float.fromhex(qv)] for i, nv, qv in rec["visited"]]
            # the recorded move leads to the next recorded root
            if r + 1 < len(c["moves"]):
                nxt, _, status = eng.next_state(roots[t:t + 1].contiguous(),
                                                torch.tensor([mv["action"]], dtype=torch.int32, device=dev))
                assert int(status[0]) == 0
                assert (nxt[0].cpu().numpy() == state_of(c["moves"][r + 1]["root"])).all()


def test_masked_softmax_prior_matches_torch(engines):
    """prior_mode 0: P = exp(log_softmax(logp[legal])) as get_valid_dist computes it."""
    from blokus_rl_amd.alphazero.batched_mcts import BatchedMCTS
    from blokus_rl_amd.boards import random_boards

    eng = engines[(20, 4, 5)]
    T = 16
    m = BatchedMCTS(eng, T, node_cap=64, child_cap=T * 64 * 1024)
    roots = random_boards(eng, T, seed0=100, max_plies=40)
    gen = torch.Generator(device=eng.device).manual_seed(0)
    logits = torch.randn((T, eng.A), generator=gen, device=eng.device) * 3.0
    logp = torch.log_softmax(logits, dim=1)
    vals = torch.zeros((T, eng.P), dtype=torch.float32, device=eng.device)
    status, _, mask = m.select(roots, None, 1.0)
    m.expand_backup(logp.contiguous(), vals, prior_mode=0)
    ids, n, q, p, counts = m.root_stats(roots)
    bits = eng.unpack_mask(mask)
    for t in range(T):
        if int(status[t]) != 1:
            continue
        K = int(counts[t])
        ref = torch.exp(torch.log_softmax(torch.masked_select(logp[t], bits[t]), dim=-1))
        assert torch.equal(ids[t, :K].long(), torch.nonzero(bits[t]).view(-1))
        torch.testing.assert_close(p[t, :K], ref, rtol=2e-6, atol=1e-7)


def test_nan_priors_flag_an_error_instead_of_faulting(engines):
    """A diverged net (NaN priors and values): no child wins the PUCT argmax, so the descent
    flags kErrIllegal and stops (status 0) — no placement, no out-of-range path record — and
    check() raises; the next expand_backup is a no-op for that tree."""
    from blokus_rl_amd.alphazero.batched_mcts import BatchedMCTS
    from blokus_rl_amd.engine import EngineError

    eng = engines[(20, 4, 5)]
    T = 2
    m = BatchedMCTS(eng, T, node_cap=64, child_cap=T * 64 * 1024)
    roots = eng.init_states(T)
    logp = torch.full((T, eng.A), float("nan"), dtype=torch.float32, device=eng.device)
    vals = torch.full((T, eng.P), float("nan"), dtype=torch.float32, device=eng.device)
    status, _, _ = m.select(roots, None, 1.0)
    assert status.tolist() == [1, 1]
    m.expand_backup(logp, vals, prior_mode=0)  # the roots expand with NaN priors
    status, _, _ = m.select(roots, None, 1.0)
    assert status.tolist() == [0, 0]
    m.expand_backup(logp, vals, prior_mode=0)
    torch.cuda.synchronize()
    with pytest.raises(EngineError):
        m.check()
