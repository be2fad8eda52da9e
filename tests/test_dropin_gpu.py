"""The drop-in boundary classes on the GPU engine, read like the reference's own call sites:
ColosseumBlokusGameWrapper (blokus_wrapper.py), MCTS (mcts.py) driven exactly as
trainer._self_play / MCTSPlayer drive it, BlokusNNetWrapper.predict / predict_batch, the
arena and the Coach's self-play."""
import importlib.util
import os
import types

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from mcts_golden_util import load_cases, prior_value, state_of, unhex
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def _hp(**kw):
    from blokus_rl_amd.hparams import AlphaZeroHparams
    return AlphaZeroHparams(**kw)


@pytest.fixture(scope="module")
def game20():
    from blokus_rl_amd.colossumrl import ColosseumBlokusGameWrapper
    return ColosseumBlokusGameWrapper(_hp(board_size=20, number_of_players=4))


@pytest.fixture(scope="module")
def game7():
    from blokus_rl_amd.colossumrl import ColosseumBlokusGameWrapper
    return ColosseumBlokusGameWrapper(_hp(board_size=7, number_of_players=2))


def test_game_wrapper_matches_oracle(game20):
    o = Oracle(20, 4, 5)
    g = game20
    assert g.get_action_size() == 30433 and g.get_observation_size() == [8, 20, 20]
    s, p = g.get_init_board()
    assert p == 0 and (s == o.init_state()).all()
    rng = np.random.default_rng(0)
    while g.get_game_ended(s) is None:
        mask = g.get_valid_moves(s, p)
        assert mask.dtype == np.float64 and mask.shape == (30433,)
        ids = np.nonzero(mask)[0]
        assert (ids == o.legal_ids(s)).all()
        other = (p + 1) % 4
        assert (np.nonzero(g.get_valid_moves(s, other))[0] == o.legal_ids(s, other)).all()
        obs, m2 = g.get_observation(s, p)
        assert (obs == o.observe(s)).all() and (m2 == mask).all()
        assert g.string_representation(s) == o.hash(s)
        a = int(rng.choice(ids))
        s2, p2 = g.get_next_state(s, p, a)
        ref, refp = o.next_state(s, a)
        assert (s2 == ref).all() and p2 == refp
        # strings round-trip through the action dicts (blokus_wrapper.py:102)
        s3, _ = g.get_next_state(s, p, g.action_move_dict[a])
        assert (s3 == s2).all()
        s, p = s2, p2
    assert (g.get_game_ended(s) == o.game_ended(s)).all()
    with pytest.raises(KeyError):
        g.get_next_state(s, p, "no-such-move")


def test_illegal_id_raises(game20):
    s, p = game20.get_init_board()
    with pytest.raises(ValueError):
        game20.get_next_state(s, p, 5)


class _StubNet:
    """Reference-style predict(obs, mask) -> (p, v) from the golden prior function."""

    def __init__(self, game, o):
        self.game, self.o = game, o
        self.last = None

    def predict(self, obs, mask):
        ids = np.nonzero(mask)[0]
        # recover the leaf state's hash: the engine's obs rows + mask are not enough, so the
        # stub keeps a board->hash map filled through the game wrapper's observation
        h = self.o.hash(self._state_from_obs(obs))
        p, v = prior_value(h, len(ids), self.o.P)
        return p, v

    def _state_from_obs(self, obs):
        P, N = self.o.P, self.o.N
        cells = np.zeros((N, N), dtype=np.int8)
        for k in range(P):
            cells[obs[k] > 0.5] = k + 1
        tm = int(np.argmax([obs[P + k, 0, 0] for k in range(P)]))
        # hash is board-only: pieces / to_move / flags do not enter it
        return self.o.make_state(cells, [0, 0, 0, 0], tm)


@pytest.mark.parametrize("k", [0, 3, 6, 7, 8])
def test_dropin_mcts_matches_reference(k, game20, game7):
    """MCTS.simulate / get_distribution called the way trainer._self_play calls them, with the
    reference-style predict() stub; distributions and root visit counts equal the golden
    vectors of the reference mcts.py."""
    from blokus_rl_amd.alphazero.mcts import MCTS
    from blokus_rl_amd.colossumrl import ColosseumBlokusGameWrapper

    case = load_cases()[k]
    preset = tuple(case["preset"])
    g = {(20, 4, 5): game20, (7, 2, 5): game7}.get(preset) or ColosseumBlokusGameWrapper(
        _hp(board_size=preset[0], number_of_players=preset[1], max_piece_cells=preset[2]))
    o = Oracle(*preset)
    tree = MCTS(g, _StubNet(g, o), node_cap=4096)
    for mv in case["moves"]:
        s = state_of(mv["root"])
        p = g.to_move(s)
        for _ in range(mv["sims"]):
            tree.simulate(s, p, cpuct=case["cpuct"], epsilon_fix=case.get("epsilon_fix", True))
        d1 = tree.get_distribution(s, 1)
        d0 = tree.get_distribution(s, 0)
        assert [int(x[0]) for x in d1[:, 0]] == mv["ids"]
        assert list(d1[:, 1]) == unhex(mv["dist_T1"])
        assert list(d0[:, 1]) == unhex(mv["dist_T0"])


@pytest.mark.parametrize("math,blocks", [("x3", 2), ("f32", 2), ("x3", 5), ("f32", 5)])
def test_predict_batch_matches_reference_predict(game20, math, blocks, monkeypatch):
    """The device leaf path (BN-folded net in one HIP launch: k_leafnet_x3, or the exact-f32
    kernels with BK_NET_MATH=f32) and the batch-1 predict() drop-in against the reference
    predict() golden rows (make_net_golden.py: the reference module on the CPU in fp32). Both
    sides carry fp32 rounding (different summation orders, BN folded vs not), so the bound is
    fp32-class: priors within 1e-5 relative (+1e-9), values within 1e-5 (|v| <= 1)."""
    monkeypatch.setenv("BK_NET_MATH", math)
    from blokus_rl_amd.neural_network import BlokusNNetWrapper

    spec = importlib.util.spec_from_file_location("mng", os.path.join(GOLDEN, "make_net_golden.py"))
    mng = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mng)
    G = np.load(os.path.join(GOLDEN, "net_golden.npz"))
    nn = BlokusNNetWrapper(game20, _hp(num_res_blocks=blocks), device=game20.device)
    sfx = "" if blocks == 2 else "b5"  # golden rows of the 2-block and the config-3 (5-block) net
    sd = nn.model.state_dict()
    nn.model.load_state_dict({k: v.to(game20.device) for k, v in mng.det_state_dict({k: v.shape for k, v in sd.items()}).items()})
    worst = [0.0, 0.0]
    n20 = sum(1 for k in G.files if k.startswith("obs20_"))  # mid-game, empty and spread boards
    for i in range(n20):
        obs = torch.from_numpy(G[f"obs20_{i}"]).unsqueeze(0).to(game20.device)
        lp, v = nn.predict_batch(obs)
        ids = torch.from_numpy(G[f"ids20_{i}"]).long().to(game20.device)
        p = torch.softmax(lp[0, ids].double(), dim=0).cpu().numpy()
        pg = G[f"p20{sfx}_{i}"].astype(np.float64)
        worst[0] = max(worst[0], float(np.max(np.abs(p - pg) / pg)))
        worst[1] = max(worst[1], float(np.max(np.abs(v[0].cpu().numpy() - G[f"v20{sfx}_{i}"]))))
        np.testing.assert_allclose(p, pg, rtol=1e-5, atol=1e-9)
        np.testing.assert_allclose(v[0].cpu().numpy(), G[f"v20{sfx}_{i}"], atol=1e-5)
        pr, vr = nn.predict(G[f"obs20_{i}"], np.isin(np.arange(30433), G[f"ids20_{i}"]).astype(np.float64))
        np.testing.assert_allclose(pr, pg, rtol=1e-5, atol=1e-9)
        np.testing.assert_allclose(vr, G[f"v20{sfx}_{i}"], atol=1e-5)
    print(f"predict {math} blocks={blocks}: max rel err p {worst[0]:.2e}, max abs err v {worst[1]:.2e}")


def test_arena_and_players_7x7(game7):
    from blokus_rl_amd.alphazero.arena import play_match
    from blokus_rl_amd.neural_network import BlokusNNetWrapper
    from blokus_rl_amd.players import MCTSPlayer, RandomPlayer

    np.random.seed(0)
    nn = BlokusNNetWrapper(game7, _hp(board_size=7, number_of_players=2, model_type="dumbnet"), device=game7.device)
    players = [MCTSPlayer(game7, nn, 20), RandomPlayer(game7)]
    scores, items = play_match(game7, players, games_num=2, permute=True)
    assert scores.shape == (2,) and len(items) == 2
    for it in items:
        assert sorted(it["scores"].tolist()) in ([-1.0, 3.0], [1.0, 1.0])


def test_coach_self_play_7x7():
    from blokus_rl_amd.alphazero.trainer import AlphaZeroTrainer

    np.random.seed(42)
    hp = _hp(board_size=7, number_of_players=2, model_type="resnet", num_res_blocks=1, num_mcts_sims=8,
             games_per_gpu=4, num_eps=4, epochs=1, batch_size=16, checkpoint_dir="/tmp/bkaz/ck", data_dir="/tmp/bkaz/data")
    tr = AlphaZeroTrainer(hp)
    data = tr._self_play(1.0)  # the reference episode, one game, np.random driven
    assert len(data) > 0 and all(d[3] is not None for d in data)
    for obs, mask, pi, z in data:
        assert obs.shape == (4, 7, 7) and mask.shape == (2522,)
        assert abs(float(pi.sum()) - 1.0) < 1e-4 and len(pi) == int(mask.sum())
    batched = tr.self_play_batched(4)
    assert len(batched) > 0
    loss = tr._train_epochs(batched)
    assert np.isfinite(loss)


def test_coach_device_iteration_7x7(tmp_path):
    """One device-path iteration: batched self-play -> packed shard on disk -> replay window ->
    learner epochs -> batched arena compare -> Elo -> checkpoint."""
    from blokus_rl_amd import replay_io as rio
    from blokus_rl_amd.alphazero.trainer import AlphaZeroTrainer

    hp = _hp(board_size=7, number_of_players=2, model_type="resnet", num_res_blocks=1, num_mcts_sims=6,
             games_per_gpu=6, num_eps=6, epochs=2, batch_size=32, compare_arena_games=2,
             checkpoint_dir=str(tmp_path / "ck"), data_dir=str(tmp_path / "data"))
    tr = AlphaZeroTrainer(hp)
    tr.iteration = 1
    s = tr.run_iteration_device()
    assert s["examples"] > 0 and s["replay_rows"] == s["examples"] and np.isfinite(s["loss"])
    assert len(s["arena_scores"]) == 2 and s["elo"] != 1000 or s["arena_scores"][0] == 0
    shards = rio.list_shards(hp.data_dir)
    assert len(shards) == 1 and rio.read_header(shards[0])["rows"] == s["examples"]
    assert (tmp_path / "ck" / "checkpoint_1.pth.tar").exists()


@pytest.mark.parametrize("k", [0, 1, 2, 3, 4])
def test_dropin_self_play_matches_reference_episode(k, game20, game7):
    """AlphaZeroTrainer._self_play (the drop-in episode over the GPU MCTS) against whole
    episodes of the reference trainer.py:92-137 (tests/golden/make_selfplay_golden.py): with the
    same np.random seed and the golden prior stub, every ply's float32 pi is bit-identical, the
    sampled actions agree (the mask/obs rows follow from them) and z equals the golden scores."""
    from blokus_rl_amd.alphazero.trainer import AlphaZeroTrainer
    from blokus_rl_amd.colossumrl import ColosseumBlokusGameWrapper
    from mcts_golden_util import load_episodes, pi_of

    ep = load_episodes()[k]
    preset = tuple(ep["preset"])
    g = {(20, 4, 5): game20, (7, 2, 5): game7}.get(preset) or ColosseumBlokusGameWrapper(
        _hp(board_size=preset[0], number_of_players=preset[1], max_piece_cells=preset[2]))
    o = Oracle(*preset)
    tr = object.__new__(AlphaZeroTrainer)
    tr.hparams = _hp(board_size=preset[0], number_of_players=preset[1], num_mcts_sims=ep["sims"], cpuct=ep["cpuct"])
    tr.game, tr.nnet = g, _StubNet(g, o)
    np.random.seed(ep["seed"])
    data = tr._self_play(ep["temperature"])
    assert len(data) == len(ep["actions"])
    s = o.init_state()
    for ply, (obs, mask, pi, z) in enumerate(data):
        assert (obs == o.observe(s)).all()
        assert (np.nonzero(mask)[0] == o.legal_ids(s)).all() and len(pi) == ep["K"][ply]
        assert pi.dtype == np.float32 and pi.tobytes() == pi_of(ep["pi"][ply]).tobytes(), f"ply {ply}"
        assert list(z) == ep["z"]
        s, _ = o.next_state(s, ep["actions"][ply])
    assert o.game_ended(s).tolist() == ep["z"]
