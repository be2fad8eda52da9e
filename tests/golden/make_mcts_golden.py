"""Golden MCTS vectors from the reference's own search code.

Run here (never on the GPU box): `python tests/golden/make_mcts_golden.py`.
It loads the reference `MCTS` class by file path from /root/reference/blokus_rl/alphazero/mcts.py
(it needs only math + numpy) and drives it with
  * a Game object exposing the reference wrapper's interface (blokus_wrapper.py:52-218) backed by
    the C oracle (oracle/blokus_oracle.c), board-keyed by the engine's 64-bit board hash;
  * a stub net whose `predict` returns deterministic priors/values, `prior_value(hash, K, P)`
    below: p as float32 (what BlokusNNetWrapper.predict returns, neural_network.py:92-110) and v
    as float64 holding float32-rounded values, so the reference's Q arithmetic is float64 under
    numpy 2 exactly as under its pinned numpy 1.25 (setup.py).
For each case it runs `num_sims` simulations from the root, records the full tree (every node's
state, child ids, N, Q, P), get_distribution at T=1 and T=0, then plays the T=0 move and repeats
on the reused tree (trainer.py:95 keeps one tree per game). Output: tests/golden/mcts_golden.json
(data only: states, ids, counts, float64 values as hex).
"""
import base64
import importlib.util
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.oracle import Oracle  # noqa: E402

REF_MCTS = "/root/reference/blokus_rl/alphazero/mcts.py"


def prior_value(h: int, K: int, P: int):
    """Deterministic stand-in for the policy/value net, shared with tests/test_mcts_gpu.py."""
    rng = np.random.default_rng(h & 0x7FFFFFFFFFFFFFFF)
    x = rng.standard_normal(K).astype(np.float32)
    e = np.exp(x - x.max()).astype(np.float32)
    p = (e / e.sum()).astype(np.float32)
    v = rng.uniform(-1.0, 1.0, P).astype(np.float32)
    return p, v


class OracleGame:
    """The reference Game interface (blokus_wrapper.py) over the oracle."""

    def __init__(self, o: Oracle):
        self.o = o
        self.last_state = None

    def get_action_size(self):
        return self.o.A

    def string_representation(self, s):
        return self.o.hash(s)

    def get_next_state(self, s, player, action):
        s2, p2 = self.o.next_state(s, int(action))
        return s2, p2

    def get_game_ended(self, s):
        return self.o.game_ended(s)

    def get_valid_moves(self, s, player):
        mask = np.zeros(self.o.A)
        mask[self.o.legal_ids(s, player)] = 1
        return mask

    def get_observation(self, s, player):
        self.last_state = s
        return self.o.observe(s), self.get_valid_moves(s, player)


class StubNet:
    def __init__(self, game: OracleGame):
        self.game = game

    def predict(self, obs, mask):
        s = self.game.last_state
        K = int(mask.sum())
        p, v = prior_value(self.game.o.hash(s), K, self.game.o.P)
        return p, v.astype(np.float64)


def load_reference_mcts():
    spec = importlib.util.spec_from_file_location("ref_mcts", REF_MCTS)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.MCTS


def b64(st: np.ndarray) -> str:
    return base64.b64encode(st.tobytes()).decode()


def dump_tree(game: OracleGame, tree, root, max_nodes=48):
    """Walk the reference tree from the root (breadth first) and record every node."""
    nodes = []
    seen = set()
    frontier = [root]
    while frontier and len(nodes) < max_nodes:
        nxt = []
        for s in frontier:
            h = game.string_representation(s)
            if h in seen or h not in tree.tree:
                continue
            seen.add(h)
            stats = tree.tree[h]
            ids = [int(a[0]) for a in stats[:, 0]]
            N = [int(x) for x in stats[:, 1]]
            # sparse: (child index, N, Q) of visited children; ids are the ascending legal ids
            # and P = prior_value(hash, K), both recomputable from the state
            visited = [[i, N[i], float(stats[i, 2]).hex()] for i in range(len(N)) if N[i] > 0]
            nodes.append({"state": b64(s), "K": len(ids), "visited": visited})
            for a, n in zip(ids, N):
                if n > 0:
                    nxt.append(game.get_next_state(s, None, a)[0])
        frontier = nxt
    return nodes


def run_case(MCTS, preset, root, num_sims, cpuct, moves, epsilon_fix=True):
    o = Oracle(*preset)
    game = OracleGame(o)
    net = StubNet(game)
    tree = MCTS(game, net)
    s = root
    out_moves = []
    for _ in range(moves):
        if o.game_ended(s) is not None:
            break
        player = Oracle.to_move(s)
        for _ in range(num_sims):
            tree.simulate(s, player, cpuct=cpuct, epsilon_fix=epsilon_fix)
        d1 = tree.get_distribution(s, 1)
        d0 = tree.get_distribution(s, 0)
        a = int(d0[int(np.argmax(d0[:, 1])), 0][0])
        out_moves.append({
            "root": b64(s),
            "sims": num_sims,
            "P": [float(x).hex() for x in tree.tree[game.string_representation(s)][:, 3]],
            "dist_T1": [float(x).hex() for x in d1[:, 1]],
            "dist_T0": [float(x).hex() for x in d0[:, 1]],
            "ids": [int(x[0]) for x in d1[:, 0]],
            "nodes": dump_tree(game, tree, s),
            "action": a,
        })
        s, _ = o.next_state(s, a)
    return {"preset": list(preset), "cpuct": cpuct, "epsilon_fix": epsilon_fix, "moves": out_moves}


def main():
    MCTS = load_reference_mcts()
    cases = []
    o20, o7 = Oracle(20, 4, 5), Oracle(7, 2, 5)
    # (preset, root, sims, cpuct, moves)
    specs = [
        ((20, 4, 5), o20.init_state(), 40, 1, 2),
        ((20, 4, 5), o20.random_board(5, 30), 60, 1, 2),
        ((20, 4, 5), o20.random_board(17, 60), 60, 2, 2),
        ((7, 2, 5), o7.init_state(), 120, 1, 3),
        ((7, 2, 5), o7.random_board(3, 4), 150, 1, 3),
        ((7, 2, 5), o7.random_board(9, 6), 150, 3, 2),
        ((7, 2, 4), Oracle(7, 2, 4).init_state(), 100, 1, 2),
        # simulate(..., epsilon_fix=False): sqrt(N.sum() + 0) at the root (mcts.py:43)
        ((20, 4, 5), o20.init_state(), 40, 1, 2, False),
        ((7, 2, 5), o7.random_board(3, 4), 150, 2, 2, False),
    ]
    for k, (preset, root, sims, cpuct, moves, *eps) in enumerate(specs):
        c = run_case(MCTS, preset, root, sims, cpuct, moves, *eps)
        nn = sum(len(m["nodes"]) for m in c["moves"])
        print(f"case {k}: preset {preset} sims {sims} cpuct {cpuct} eps_fix {c['epsilon_fix']} "
              f"moves {len(c['moves'])} nodes {nn}")
        cases.append(c)
    out = {
        "generator": "tests/golden/make_mcts_golden.py driving /root/reference/blokus_rl/alphazero/mcts.py",
        "prior": "prior_value(hash, K, P) in make_mcts_golden.py",
        "cases": cases,
    }
    fp = os.path.join(HERE, "mcts_golden.json")
    with open(fp, "w", encoding="utf-8") as f:
        json.dump(out, f, separators=(",", ":"))
    print(fp, os.path.getsize(fp), "bytes")


if __name__ == "__main__":
    main()
