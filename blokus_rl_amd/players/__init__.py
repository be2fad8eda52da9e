"""Players of the arena API (blokus_rl/players/*.py): update_state(s, p) -> (s', p'), reset()."""
from __future__ import annotations

from abc import ABC, abstractmethod

import numpy as np


class Player(ABC):
    @abstractmethod
    def update_state(self, s, current_player):
        raise NotImplementedError

    @abstractmethod
    def reset(self):
        raise NotImplementedError


class MCTSPlayer(Player):
    """players/mcts_player.py:8-28: `simulations` searches, then the T=0 (argmax) move."""

    def __init__(self, game, nn, simulations):
        from ..alphazero.mcts import MCTS, node_cap_for

        self.game, self.nn, self.simulations = game, nn, simulations
        self._mcts_cls = MCTS
        self._node_cap = max(node_cap_for(game), node_cap_for(game, simulations))
        self.tree = MCTS(game, nn, node_cap=self._node_cap)

    def update_state(self, s, current_player):
        for _ in range(self.simulations):
            self.tree.simulate(s, current_player)
        dist = self.tree.get_distribution(s, 0)
        a = dist[np.argmax(dist[:, 1]), 0]
        return self.game.get_next_state(s, current_player, a[0])

    def reset(self):
        self.tree = self._mcts_cls(self.game, self.nn, node_cap=self._node_cap)

    def __str__(self):
        return "MCTSPlayer"


class RandomPlayer(Player):
    """players/random_player.py:5-24."""

    def __init__(self, game):
        self.game = game

    def update_state(self, s, current_player):
        return self.game.get_next_state(s, current_player, self.game.get_sample_move(s))

    def reset(self):
        return

    def __str__(self):
        return "RandomPlayer"


class HumanPlayer(Player):
    """players/human_player.py:5-44 (stdin)."""

    def __init__(self, game):
        self.game = game

    def update_state(self, s, current_player):
        actions = self.game.get_valid_actions_for_human_player(s, current_player)
        self.game.display(s)
        for i, a in enumerate(actions):
            print(f"{i}: {a}")
        while True:
            a = input("Enter move: ")
            if a.isdigit() and int(a) in range(len(actions)):
                break
            print("Invalid move. Try again.")
        return self.game.get_next_state(s, current_player, actions[int(a)])

    def reset(self):
        return

    def __str__(self):
        return "HumanPlayer"
