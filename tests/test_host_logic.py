"""Host-side sizing logic that needs no GPU."""
from types import SimpleNamespace

from blokus_rl_amd.alphazero.selfplay import SelfPlay


def test_node_cap_bounds_a_whole_game():
    # 20x20, 4 players, 21 pieces: at most 84 plies, each adding <= num_sims nodes to the tree
    eng = SimpleNamespace(num_pieces=21, P=4)
    assert SelfPlay.max_game_plies(eng) == 84
    assert SelfPlay.node_cap_for(eng, 100) == 8401  # above the old fixed 8192
    assert SelfPlay.node_cap_for(SimpleNamespace(num_pieces=9, P=2), 25) == 451
