"""The pure-Python MCTS restatement (oracle/oracle.py MCTSOracle) against golden vectors
produced by the reference's own blokus_rl/alphazero/mcts.py (tests/golden/make_mcts_golden.py):
root N, Q (float64, bit-exact), P, every recorded node's visited children, and
get_distribution at T=1 / T=0, across moves on a reused tree."""
import numpy as np
import pytest

from mcts_golden_util import load_cases, prior_value, state_of, unhex
from oracle.oracle import MCTSOracle, Oracle

CASES = load_cases()


@pytest.mark.parametrize("k", range(len(CASES)))
def test_mcts_oracle_matches_reference(k):
    case = CASES[k]
    o = Oracle(*case["preset"])

    def evaluate(s, player):
        ids = o.legal_ids(s, player)
        p, v = prior_value(o.hash(s), len(ids), o.P)
        return ids, p, v.astype(np.float64)

    m = MCTSOracle(o, evaluate)
    for mv in case["moves"]:
        root = state_of(mv["root"])
        for _ in range(mv["sims"]):
            r = m.simulate(root, cpuct=case["cpuct"], epsilon_fix=case.get("epsilon_fix", True))
        ids, d1 = m.get_distribution(root, 1)
        _, d0 = m.get_distribution(root, 0)
        assert ids.tolist() == mv["ids"]
        assert d1.tolist() == unhex(mv["dist_T1"])
        assert d0.tolist() == unhex(mv["dist_T0"])
        node = m.tree[o.hash(root)]
        assert node["P"] == unhex(mv["P"])
        for rec in mv["nodes"]:
            nd = m.tree[o.hash(state_of(rec["state"]))]
            assert len(nd["N"]) == rec["K"]
            got = [[i, nd["N"][i], nd["Q"][i]] for i in range(rec["K"]) if nd["N"][i] > 0]
            assert got == [[i, n, float.fromhex(q)] for i, n, q in rec["visited"]]
    TERMINAL_HITS[k] = m.terminal_hits


TERMINAL_HITS = {}


def test_golden_cases_reach_terminal_leaves():
    """At least one golden case exercises terminal leaves (one-hot scores backed up)."""
    if len(TERMINAL_HITS) < len(CASES):
        pytest.skip("run with the parametrized cases")
    assert sum(TERMINAL_HITS.values()) > 0, TERMINAL_HITS


EPISODES = None


def _episodes():
    global EPISODES
    if EPISODES is None:
        from mcts_golden_util import load_episodes
        EPISODES = load_episodes()
    return EPISODES


@pytest.mark.parametrize("k", range(5))
def test_oracle_episode_matches_reference_self_play(k):
    """A whole reference self-play episode (trainer.py:92-137, golden from
    make_selfplay_golden.py) restated over MCTSOracle: the same legacy np.random stream
    (np.random.seed, Dirichlet(1) root noise at weight 0.25, np.random.choice on the float32
    pi) gives the same actions, bit-identical float32 pi per ply and the same final scores."""
    from mcts_golden_util import pi_of
    ep = _episodes()[k]
    o = Oracle(*ep["preset"])

    def evaluate(s, player):
        ids = o.legal_ids(s, player)
        p, v = prior_value(o.hash(s), len(ids), o.P)
        return ids, p, v.astype(np.float64)

    m = MCTSOracle(o, evaluate)
    np.random.seed(ep["seed"])
    s = o.init_state()
    root = True
    for ply, a_ref in enumerate(ep["actions"]):
        assert o.game_ended(s) is None
        for _ in range(ep["sims"]):
            m.simulate(s, cpuct=ep["cpuct"])
        ids, d = m.get_distribution(s, ep["temperature"])
        if root:
            noise = np.random.dirichlet(np.array(1 * np.ones_like(d.astype(np.float32))))
            d = d * 0.75 + noise * 0.25
            root = False
        pi = d.astype(np.float32)
        assert len(ids) == ep["K"][ply] == len(o.legal_ids(s))
        assert pi.tobytes() == pi_of(ep["pi"][ply]).tobytes(), f"ply {ply}"
        a = int(ids[np.random.choice(len(d), p=pi)])
        assert a == a_ref, f"ply {ply}"
        s, _ = o.next_state(s, a)
    assert o.game_ended(s).tolist() == ep["z"]
