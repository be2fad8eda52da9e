"""Batched arena == the reference-order sequential arena (arena.py:10-87 with
MCTSPlayer seats, players/mcts_player.py:8-28) on the drop-in classes: same per-game scores,
same accumulated scores, for uninformed (DumbNet) and ResNet seats, 7x7 and 20x20."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _hp(**kw):
    from blokus_rl_amd.hparams import AlphaZeroHparams
    return AlphaZeroHparams(**kw)


def _game(n, p):
    from blokus_rl_amd.colossumrl import ColosseumBlokusGameWrapper
    return ColosseumBlokusGameWrapper(_hp(board_size=n, number_of_players=p))


def _nn(game, model_type, seed=0, blocks=1):
    from blokus_rl_amd.neural_network import BlokusNNetWrapper
    torch.manual_seed(seed)
    n, p = game.board_size, game.number_of_players
    return BlokusNNetWrapper(game, _hp(board_size=n, number_of_players=p, model_type=model_type,
                                       num_res_blocks=blocks), device=game.device)


def _both(game, players, games, permute):
    from blokus_rl_amd.alphazero.arena import play_match
    from blokus_rl_amd.alphazero.batched_arena import play_match_batched

    s_seq, items_seq = play_match(game, players, games_num=games, permute=permute)
    s_bat, items_bat = play_match_batched(game, players, games_num=games, permute=permute)
    return s_seq, items_seq, s_bat, items_bat


@pytest.mark.parametrize("n,p,games,sims", [(7, 2, 4, (12, 7)), (20, 4, 3, (3, 4, 2, 3))])
def test_batched_arena_uninformed_equals_sequential(n, p, games, sims):
    from blokus_rl_amd.players import MCTSPlayer

    game = _game(n, p)
    dumb = _nn(game, "dumbnet")
    players = [MCTSPlayer(game, dumb, s) for s in sims]
    s_seq, it_seq, s_bat, it_bat = _both(game, players, games, permute=True)
    for a, b in zip(it_seq, it_bat):
        np.testing.assert_array_equal(a["scores"], b["scores"])
    np.testing.assert_array_equal(s_seq, s_bat)


def test_batched_arena_two_nets_equals_sequential():
    """The arena-compare shape: a new net against copies of the previous one (trainer.py:222-271)."""
    from blokus_rl_amd.players import MCTSPlayer

    game = _game(7, 2)
    new, old = _nn(game, "resnet", 1), _nn(game, "resnet", 2)
    players = [MCTSPlayer(game, new, 10), MCTSPlayer(game, old, 10)]
    s_seq, it_seq, s_bat, it_bat = _both(game, players, 4, permute=True)
    same = sum(bool(np.array_equal(a["scores"], b["scores"])) for a, b in zip(it_seq, it_bat))
    assert same == len(it_seq), (s_seq, s_bat)


def test_batched_arena_rejects_non_mcts_players():
    from blokus_rl_amd.alphazero.batched_arena import play_match_batched
    from blokus_rl_amd.players import RandomPlayer

    game = _game(7, 2)
    with pytest.raises(TypeError):
        play_match_batched(game, [RandomPlayer(game), RandomPlayer(game)], 1)


def test_batched_arena_plays_full_games():
    """Games run to the end: every game over, plies in the range of real games, one winner row."""
    from blokus_rl_amd.alphazero.batched_arena import ArenaSeat, BatchedArena
    from blokus_rl_amd.engine import W_PLY

    game = _game(20, 4)
    arena = BatchedArena(game.engine, [ArenaSeat(None, 2) for _ in range(4)])
    scores, per_game, states = arena.play(4, permute=True)
    ended, _ = game.engine.game_ended(states)
    assert bool(ended.all())
    plies = states.view(torch.int32)[:, W_PLY].cpu().numpy()
    assert (plies >= 40).all() and (plies <= 84).all(), plies
    for row in per_game:
        assert sorted(row.tolist()) in ([-1, -1, -1, 3], [-1, -1, 1, 1], [-1, 1, 1, 1], [1, 1, 1, 1])
    assert scores.sum() == per_game.sum()
