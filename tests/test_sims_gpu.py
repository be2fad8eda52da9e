"""The fused leaf step (bk_mcts_leaf_step: sparse policy head + expand/backup + the next descent in
one launch) against the per-stage launches it fuses (k_leaf_logits -> k_expand_backup ->
k_select): the trees, counters and leaf outputs come out bitwise identical. Also the captured
simulation graph (SelfPlay.sim_graph_sims) against eager launches."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _leaf_model(eng, blocks=2, seed=0):
    from blokus_rl_amd.nets import LeafResNet, ResNet

    torch.manual_seed(seed)
    net = ResNet(eng.N, eng.P, eng.A, blocks).cuda().eval()
    return LeafResNet(net, normalize=False, features=True).eval()


@pytest.mark.parametrize("N,T,sims,overlap,skip0", [(20, 12, 9, "1", "1"), (20, 12, 9, "0", "1"), (14, 7, 6, "1", "1"),
                                                    (20, 64, 40, "1", "1"), (20, 64, 40, "1", "0")])
def test_leaf_step_matches_stagewise(N, T, sims, overlap, skip0, monkeypatch):
    """bk_mcts_leaf_step (policy head + expand/backup + the next descent in one launch; overlap 1
    = k_leaf_step_ov, the default, whose wave 0 backs up and descends while the other waves
    compute the logits) against k_leaf_logits -> k_expand_backup -> k_select: the same trees,
    counters, leaf states and observations, bitwise — with the sparse head's zero-feature skip
    (BK_LEAF_SKIP0=1, the default: W float4s of four zero features not loaded) and without it."""
    monkeypatch.setenv("BK_STEP_OVERLAP", overlap)
    monkeypatch.setenv("BK_LEAF_SKIP0", skip0)
    from blokus_rl_amd.alphazero.batched_mcts import BatchedMCTS
    from blokus_rl_amd.boards import random_boards
    from blokus_rl_amd.engine import Engine

    eng = Engine(N, 4, 5)
    model = _leaf_model(eng)
    roots = random_boards(eng, T, seed0=11, max_plies=24 if N == 20 else 12)
    active = torch.ones(T, dtype=torch.int32, device=eng.device)
    active[T // 3] = 0
    kw = dict(node_cap=sims + 8, child_cap=T * (sims + 8) * 700)
    m1, m2 = BatchedMCTS(eng, T, **kw), BatchedMCTS(eng, T, **kw)
    po = model.f.policy_out
    w, b = po.weight.detach().contiguous(), po.bias.detach().contiguous()
    _, obs1, _ = m1.select(roots, active, 1.5)
    _, obs2, _ = m2.select(roots, active, 1.5)
    for i in range(sims):
        pf1, v1 = (t.contiguous() for t in model(obs1))
        pf2, v2 = (t.contiguous() for t in model(obs2))
        assert torch.equal(pf1, pf2) and torch.equal(v1, v2)
        m1.leaf_logits(pf1, w, b)
        m1.expand_backup(None, v1, 2)
        last = i == sims - 1
        if not last:
            st1, obs1, mk1 = m1.select(roots, active, 1.5)
        r = m2.leaf_step(pf2, w, b, v2, None if last else roots, active, 1.5)
        if not last:
            st2, obs2, mk2 = r
            assert torch.equal(st1, st2) and torch.equal(obs1, obs2)
            ok = st1 == 1
            assert torch.equal(mk1[ok], mk2[ok])
    c1, c2 = m1.check(), m2.check()
    assert c1 == c2 and c1["expanded"] > 0
    for x, y in zip(m1.root_stats(roots, active), m2.root_stats(roots, active)):
        assert torch.equal(x, y)


@pytest.mark.parametrize("gsims", [None, 10])
def test_selfplay_plies_match_eager(monkeypatch, gsims):
    """The default play_ply path (the captured simulation graph: the whole ply in one graph, or 10
    per graph + eager rest) gives the plies of launching every stage eagerly."""
    from blokus_rl_amd.alphazero.selfplay import SelfPlay
    from blokus_rl_amd.engine import Engine
    from blokus_rl_amd.nets import ResNet

    eng = Engine(20, 4, 5)

    def run(g):
        monkeypatch.setenv("BK_SIM_GRAPH", g)
        torch.manual_seed(0)
        model = ResNet(20, 4, eng.A, num_res_blocks=2).to(eng.device).eval()
        sp = SelfPlay(eng, model, 6, num_sims=13, node_cap=256, seed=5, continuous=True,
                      sim_graph_sims=gsims if g == "1" else None)
        for _ in range(3):
            sp.play_ply()
        _, n, q, p, k = sp.mcts.root_stats(sp.roots)
        return (sp.roots.clone(), n, q, p, k), sp.mcts.check()

    ref, cref = run("0")
    got, cgot = run("1")
    for x, y in zip(ref, got):
        assert torch.equal(x, y)
    assert cref == cgot


def test_dumbnet_plies_match_eager(monkeypatch):
    from blokus_rl_amd.alphazero.selfplay import SelfPlay
    from blokus_rl_amd.engine import Engine
    from blokus_rl_amd.nets import DumbNet

    eng = Engine(7, 2, 5)

    def run(g):
        monkeypatch.setenv("BK_SIM_GRAPH", g)
        sp = SelfPlay(eng, DumbNet(7, 2, eng.A), 16, num_sims=24, node_cap=2048, seed=3)
        for _ in range(4):
            sp.play_ply()
        _, n, q, p, k = sp.mcts.root_stats(sp.roots, sp.active)
        return (sp.roots.clone(), n, q, k), sp.mcts.check()

    ref, cref = run("0")
    got, cgot = run("1")
    for x, y in zip(ref, got):
        assert torch.equal(x, y)
    assert cref == cgot
