"""Arena (blokus_rl/alphazero/arena.py:10-87): sequential P-seat matches, optional seat
permutations; scores[order] += the game's one-hot (-1 / 3 / 1) scores."""
from __future__ import annotations

from itertools import permutations

import numpy as np


def play_match(game, players: list, games_num: int, verbose=False, permute=False, capture_video=False):
    matches = list(permutations(np.arange(len(players)))) if permute else [np.arange(len(players))]
    items = []
    scores = np.zeros(game.get_number_of_players())
    for i in range(games_num):
        order = matches[i % len(matches)]
        for p in players:
            p.reset()
        current, frames = play_single_match(game, players, order, verbose, capture_video)
        scores[list(order)] += current
        items.append({"scores": current, "frames": frames})
    return scores, items


def play_single_match(game, players, order, verbose=False, capture_video=False):
    frames = []
    s, current_player = game.get_init_board()
    if capture_video:
        frames.append(game.render(s))
    current = None
    while current is None:
        p = order[current_player]
        if verbose:
            game.display(s)
        s, current_player = players[p].update_state(s, current_player)
        if capture_video:
            frames.append(game.render(s))
        current = game.get_game_ended(s)
    return current, frames
