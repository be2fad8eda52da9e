"""Config-3-shaped search parity: the production simulation path (one captured graph per ply:
k_select, then 100 x {k_leafnet_x3 on the leaf batch, k_leaf_step = sparse policy head + masked
softmax + expand/backup + the next descent}) on 64 trees of 20x20 boards with a 5-block ResNet,
replayed tree by tree through the CPU restatement of the reference search (oracle MCTSOracle,
mcts.py:7-99) with the GPU's own leaf evaluations handed over as is (prior_mode 1 semantics:
the float32 priors the search stored, the float32 values the net returned). Every expanded
node's N and Q (float64) and the root pi must agree bit for bit; the stored priors of EVERY
expanded node must equal an fp64 masked softmax of the policy head over the same features to
1e-5 (the oracle is handed the stored priors, so this is the independent check on them).

Leaf values are recomputed by the same net on each node's observation in 64-row batches (the
x3 kernel's rows do not depend on the batch, tests/test_leafnet_gpu.py); the priors are read
back from the trees with bk_mcts_root_stats, which looks any node up by its board key."""
import numpy as np
import pytest
import torch

from oracle.oracle import MCTSOracle, Oracle

pytestmark = pytest.mark.gpu

T, SIMS, BLOCKS = 64, 100, 5


def _dump_trees(sp, eng, o, roots_h, more=()):
    """BFS over every tree through visited children from its root (and the roots in `more`):
    {tree: {hash: (state, ids, N, Q, P)}}."""
    return _dump_forest(sp, eng, o, [[roots_h[t]] + [r[t] for r in more] for t in range(T)])


def _dump_forest(sp, eng, o, starts):
    """BFS over every tree t through visited children from each state of starts[t]."""
    trees = [dict() for _ in range(T)]
    frontier = [list(s) for s in starts]
    state_bytes = starts[0][0].shape[0]
    cap = 2048
    while any(frontier):
        q = np.zeros((T, state_bytes), dtype=np.uint8)
        act = np.zeros(T, dtype=np.int32)
        cur = [None] * T
        for t in range(T):
            while frontier[t]:
                s = frontier[t].pop()
                h = o.hash(s)
                if h in trees[t] or o.game_ended(s) is not None:
                    continue
                cur[t], q[t], act[t] = s, s, 1
                break
        if not act.any():
            break
        ids, n, qv, p, k = sp.mcts.root_stats(torch.from_numpy(q).to(eng.device),
                                              torch.from_numpy(act).to(eng.device), cap)
        ids, n, qv, p, k = (x.cpu().numpy() for x in (ids, n, qv, p, k))
        for t in range(T):
            if not act[t]:
                continue
            K = int(k[t])
            assert K > 0, f"tree {t}: a visited node is missing from the table"
            s = cur[t]
            trees[t][o.hash(s)] = (s, ids[t, :K].copy(), n[t, :K].astype(np.int64), qv[t, :K].copy(), p[t, :K].copy())
            for i in np.nonzero(n[t, :K])[0]:
                frontier[t].append(o.next_state(s, int(ids[t, i]))[0])
    return trees


def _check_priors(ev, nodes, feats):
    """Every expanded node's stored priors = the policy head's masked softmax over its legal ids,
    recomputed in float64 from the node's policy features: nodes {key: (state, ids, N, Q, P)},
    feats {key: features}."""
    W = ev.policy_w.cpu().double().numpy()
    b = ev.policy_b.cpu().double().numpy()
    assert nodes and set(nodes) <= set(feats)
    for key, (_, ids, _, _, P) in nodes.items():
        lg = W[ids] @ feats[key].astype(np.float64) + b[ids]
        e = np.exp(lg - lg.max())
        np.testing.assert_allclose(P, e / e.sum(), rtol=1e-5, atol=1e-7, err_msg=str(key))


def test_config3_search_matches_oracle_replay():
    from blokus_rl_amd.alphazero.selfplay import SelfPlay
    from blokus_rl_amd.boards import random_boards
    from blokus_rl_amd.engine import Engine
    from blokus_rl_amd.nets import ResNet, net_math

    eng = Engine(20, 4, 5)
    o = Oracle(20, 4, 5)
    torch.manual_seed(0)
    model = ResNet(20, 4, eng.A, num_res_blocks=BLOCKS).to(eng.device).eval()
    sp = SelfPlay(eng, model, T, num_sims=SIMS, seed=1)
    assert sp.evaluator.sparse and sp.evaluator.planar and sp._graph_usable()
    assert sp.sim_graph_sims == SIMS and net_math() == "x3"
    sp.roots = random_boards(eng, T, seed0=21, max_plies=48)
    sp._simulations(SIMS)
    c = sp.check()
    assert c["expanded"] + c["terminal"] == T * SIMS
    roots_h = sp.roots.cpu().numpy()
    rids, rpi, rk = (x.cpu().numpy() for x in sp.mcts.root_policy(sp.roots, sp.active, 1.0))
    trees = _dump_trees(sp, eng, o, roots_h)
    assert sum(len(tr) for tr in trees) == c["expanded"]

    # leaf values (and policy features) of every expanded node, recomputed by the same net
    ev = sp.evaluator
    keys = [(t, h) for t in range(T) for h in trees[t]]
    vals, feats = {}, {}
    for i in range(0, len(keys), T):
        chunk = keys[i:i + T]
        st = np.zeros((T, roots_h.shape[1]), dtype=np.uint8)
        for j, (t, h) in enumerate(chunk):
            st[j] = trees[t][h][0]
        pf, v = ev._forward(eng.observe(torch.from_numpy(st).to(eng.device)))
        v, pf = v.cpu().numpy(), pf.cpu().numpy()
        for j, key in enumerate(chunk):
            vals[key], feats[key] = v[j].astype(np.float64), pf[j]

    # the stored priors of every expanded node are the policy head's masked softmax
    _check_priors(ev, {(t, h): nd for t in range(T) for h, nd in trees[t].items()}, feats)

    for t in range(T):
        nodes = trees[t]

        def evaluate(s, player, t=t, nodes=nodes):
            h = o.hash(s)
            _, ids, _, _, P = nodes[h]
            assert (ids == o.legal_ids(s, player)).all()
            return ids, P, vals[(t, h)]

        m = MCTSOracle(o, evaluate)
        for _ in range(SIMS):
            m.simulate(roots_h[t], cpuct=sp.cpuct)
        assert set(m.tree) == set(nodes), t
        for h, nd in m.tree.items():
            _, ids, N, Q, _ = nodes[h]
            assert nd["N"] == N.tolist(), (t, h)
            assert nd["Q"] == Q.tolist(), (t, h)
        oids, d = m.get_distribution(roots_h[t], 1.0)
        K = int(rk[t])
        assert (rids[t, :K] == oids).all() and rpi[t, :K].tolist() == d.tolist(), t


PLIES = 3


def test_config3_tree_reuse_matches_oracle_replay():
    """The production self-play plies (SelfPlay.play_ply: the captured simulation graph with
    k_leaf_step_ov in continuous tree-reuse mode, then k_root / the fused ply tail picking each
    game's move) for PLIES plies on 64 trees at config-3 shape (20x20, 5-block net, 100 sims), the
    trees kept from ply to ply as the reference keeps one tree per episode (trainer.py:95,
    102-128). Replayed through ONE persistent MCTSOracle per tree from the same roots with the
    GPU's leaf evaluations: every node's N and float64 Q and each ply's root pi bit-exact after
    every ply."""
    from blokus_rl_amd.alphazero.selfplay import SelfPlay
    from blokus_rl_amd.boards import random_boards
    from blokus_rl_amd.engine import Engine
    from blokus_rl_amd.nets import ResNet, net_math

    eng = Engine(20, 4, 5)
    o = Oracle(20, 4, 5)
    torch.manual_seed(0)
    model = ResNet(20, 4, eng.A, num_res_blocks=BLOCKS).to(eng.device).eval()
    sp = SelfPlay(eng, model, T, num_sims=SIMS, seed=3)
    assert sp._graph_usable() and net_math() == "x3"
    sp.roots = random_boards(eng, T, seed0=41, max_plies=24)
    roots, dumps, pis = [], [], []
    for _ in range(PLIES):
        r = sp.roots.clone()
        sp.play_ply()
        sp.check()
        # early-game roots (<= 24 plies played): no game can end inside the window, so no tree is
        # reset and every root's node stays in its tree
        assert bool(sp.active.all())
        roots.append(r.cpu().numpy())
        pis.append(tuple(x.cpu().numpy() for x in sp.mcts.root_policy(r, None, 1.0)))
        # every root so far: a first-ply move drawn with Dirichlet noise may be an unvisited child
        dumps.append(_dump_trees(sp, eng, o, roots[0], roots[1:]))
    final = dumps[-1]

    ev = sp.evaluator
    keys = [(t, h) for t in range(T) for h in final[t]]
    vals, feats = {}, {}
    for i in range(0, len(keys), T):
        chunk = keys[i:i + T]
        st = np.zeros((T, roots[0].shape[1]), dtype=np.uint8)
        for j, (t, h) in enumerate(chunk):
            st[j] = final[t][h][0]
        pf, v = ev._forward(eng.observe(torch.from_numpy(st).to(eng.device)))
        v, pf = v.cpu().numpy(), pf.cpu().numpy()
        for j, key in enumerate(chunk):
            vals[key], feats[key] = v[j].astype(np.float64), pf[j]
    _check_priors(ev, {(t, h): final[t][h] for t, h in keys}, feats)

    for t in range(T):
        nodes = final[t]

        def evaluate(s, player, t=t, nodes=nodes):
            h = o.hash(s)
            _, ids, _, _, P = nodes[h]
            assert (ids == o.legal_ids(s, player)).all()
            return ids, P, vals[(t, h)]

        m = MCTSOracle(o, evaluate)
        for i in range(PLIES):
            for _ in range(SIMS):
                m.simulate(roots[i][t], cpuct=sp.cpuct)
            snap = dumps[i][t]
            assert set(m.tree) == set(snap), (t, i)
            for h, nd in m.tree.items():
                _, _, N, Q, _ = snap[h]
                assert nd["N"] == N.tolist(), (t, i, h)
                assert nd["Q"] == Q.tolist(), (t, i, h)
            oids, d = m.get_distribution(roots[i][t], 1.0)
            rids, rpi, rk = pis[i]
            K = int(rk[t])
            assert (rids[t, :K] == oids).all() and rpi[t, :K].tolist() == d.tolist(), (t, i)


TURN_PLIES = 5


def _near_terminal_roots(o):
    """Root t: a uniform-random game of the oracle (default_rng(1000 + t)) played to its end (52-64
    plies), backed up by 1 + t % 8 plies, so about half of the games end inside TURN_PLIES."""
    roots = []
    for t in range(T):
        rng = np.random.default_rng(1000 + t)
        hist = [o.init_state()]
        while o.game_ended(hist[-1]) is None:
            ids = o.legal_ids(hist[-1])
            hist.append(o.next_state(hist[-1], int(ids[int(rng.integers(len(ids)))]))[0])
        roots.append(hist[-1 - (1 + t % 8)])
    return np.stack(roots)


def test_config3_game_turnover_matches_oracle_replay():
    """Game turnover on the production path: SelfPlay(continuous=True).play_ply
    on 64 trees at config-3 shape (20x20, 5-block net, 100 sims) from near-terminal roots, so
    games end, their trees are reset (k_reset: a new MCTS per episode, trainer.py:95) and their
    slots restart from the empty board (k_ply_finish) inside the window. Each slot is replayed
    through one MCTSOracle per episode — persistent while the game runs, a fresh one for the
    restarted game — with the GPU's leaf evaluations: every node's N and float64 Q and each ply's
    root pi bit-exact at every ply, the restarted games' first plies included. The next roots are
    the oracle's next states (or the empty board after a game end), and z of every finished game,
    in the z table and in the rows of window_packed(), is the oracle's final one-hot score of that
    game (trainer.py:131-135); rows of running games carry z = 0."""
    from blokus_rl_amd.alphazero.selfplay import SelfPlay
    from blokus_rl_amd.engine import Engine
    from blokus_rl_amd.nets import ResNet, net_math
    from blokus_rl_amd.replay import unpack

    eng = Engine(20, 4, 5)
    o = Oracle(20, 4, 5)
    torch.manual_seed(0)
    model = ResNet(20, 4, eng.A, num_res_blocks=BLOCKS).to(eng.device).eval()
    sp = SelfPlay(eng, model, T, num_sims=SIMS, seed=5, continuous=True)
    assert sp._graph_usable() and net_math() == "x3"
    init = o.init_state()
    sp.roots = torch.from_numpy(_near_terminal_roots(o)).to(eng.device)
    sp.mark_window()
    episode_roots = [[r] for r in sp.roots.cpu().numpy()]  # roots of each slot's running episode
    plies = []  # per ply: roots, game ids, dumps, root pi, actions, ended scores per slot
    for i in range(TURN_PLIES):
        roots_h = sp.roots.cpu().numpy()
        gid = sp.game_id.cpu().numpy().copy()
        for t in range(T):
            if i > 0 and not (roots_h[t] == episode_roots[t][-1]).all():
                episode_roots[t].append(roots_h[t])
        sp._simulations(sp.num_sims)  # = play_ply: the simulations, then the fused ply tail
        dump = _dump_forest(sp, eng, o, episode_roots)
        pol = tuple(x.cpu().numpy() for x in sp.mcts.root_policy(sp.roots, None, 1.0))
        sp._ply_tail_fused(True)
        sp.check()
        act = sp.last_action.cpu().numpy()
        nxt_h = sp.roots.cpu().numpy()
        ends = [None] * T
        for t in range(T):
            assert act[t] >= 0, (i, t)
            s2, _ = o.next_state(roots_h[t], int(act[t]))
            ends[t] = o.game_ended(s2)
            if ends[t] is None:
                assert (nxt_h[t] == s2).all(), (i, t)
            else:
                # the finished game's z, and its slot restarted from the empty board with a new tree
                assert (nxt_h[t] == init).all(), (i, t)
                assert sp.z_table[int(gid[t])].cpu().numpy().tolist() == ends[t].tolist(), (i, t)
                episode_roots[t] = [init]
        plies.append((roots_h, gid, dump, pol, ends))
    ended = sum(e is not None for p in plies for e in p[4])
    restarted = [t for t in range(T) if any(p[4][t] is not None for p in plies[:-1])]
    assert ended >= 16 and len(restarted) >= 8, (ended, len(restarted))

    # leaf values of every node, recomputed by the same net (a value depends on the state only)
    vals, feats, states = {}, {}, {}
    for p in plies:
        for tr in p[2]:
            for h, nd in tr.items():
                states.setdefault(h, nd)
    hs = list(states)
    ev = sp.evaluator
    for j in range(0, len(hs), T):
        chunk = hs[j:j + T]
        st = np.zeros((T, init.shape[0]), dtype=np.uint8)
        for r, h in enumerate(chunk):
            st[r] = states[h][0]
        pf, v = ev._forward(eng.observe(torch.from_numpy(st).to(eng.device)))
        v, pf = v.cpu().numpy(), pf.cpu().numpy()
        for r, h in enumerate(chunk):
            vals[h], feats[h] = v[r].astype(np.float64), pf[r]
    _check_priors(ev, states, feats)

    for t in range(T):
        cur = {}

        def evaluate(s, player):
            h = o.hash(s)
            _, ids, _, _, P = cur["nodes"][h]
            assert (ids == o.legal_ids(s, player)).all()
            return ids, P, vals[h]

        m = None
        for i, (roots_h, _, dump, pol, ends) in enumerate(plies):
            nodes = cur["nodes"] = dump[t]
            if m is None:
                m = MCTSOracle(o, evaluate)
            for _ in range(SIMS):
                m.simulate(roots_h[t], cpuct=sp.cpuct)
            assert set(m.tree) == set(nodes), (t, i)
            for h, nd in m.tree.items():
                _, _, N, Q, _ = nodes[h]
                assert nd["N"] == N.tolist(), (t, i, h)
                assert nd["Q"] == Q.tolist(), (t, i, h)
            oids, d = m.get_distribution(roots_h[t], 1.0)
            rids, rpi, rk = pol
            K = int(rk[t])
            assert (rids[t, :K] == oids).all() and rpi[t, :K].tolist() == d.tolist(), (t, i)
            if ends[t] is not None:
                m = None  # the episode is over: the next ply's search starts a fresh tree (trainer.py:95)

    # the window's rows: ply-major, one per slot; z = the final score of the row's game once it ended
    buf, cap = sp.window_packed()
    rows = unpack(buf, cap)
    assert rows["states"].shape[0] == TURN_PLIES * T
    zrow = rows["z"].cpu().numpy()
    final = {}
    for p in plies:
        for t in range(T):
            if p[4][t] is not None:
                final[int(p[1][t])] = p[4][t]
    for i, p in enumerate(plies):
        for t in range(T):
            r = i * T + t
            assert (rows["states"][r].cpu().numpy() == p[0][t]).all()
            want = final.get(int(p[1][t]), np.zeros(4))
            assert zrow[r].tolist() == want.tolist(), (i, t)
