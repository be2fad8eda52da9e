"""The oracle against the reference's own pins: known answers and the recorded games.

Pins: 30433 actions on 20x20 (docs/README.md:128), 919 on 7x7 with the
<=4-cell set (docs/README.md:51), 58 first moves, and the three games the reference recorded in
docs/images/AlphaZero (decoded by tests/golden/make_gif_fixtures.py). Replaying a recording
move by move checks legality of every placement, the turn order with the skip rule, the
termination rule and the winner/scoring conversion (blokus_wrapper.py:164-186)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle.oracle import Oracle


def test_known_answers():
    o = Oracle(20, 4, 5)
    assert o.A == 30433
    assert o.num_pieces == 21
    for p in range(4):
        _, n = o.legal_mask(o.init_state(), p)
        assert n == 58
    assert Oracle(7, 2, 4).A == 919
    assert Oracle(7, 2, 5).A == 2522
    # 91 fixed orientations of the 21 pieces
    t = o.action_table()
    assert len({(int(a), int(b)) for a, b in t[:, :2]}) == 91


# Legal-move counts along the arena recording (computed by the survey's
# brute-force checker, an independent restatement).
ARENA_COUNTS = [int(x) for x in """58 58 58 58 113 113 106 182 198 244 162 362 296 286 283 443 343
335 285 569 427 422 323 644 271 638 256 586 249 614 234 469 102 429 161 470 62 358 170 330 57 217
64 165 64 100 18 98 101 92 2 31 28 13 3 10 8 4 1 3 1""".split()]


def _find_action(o: Oracle, cells_of_id: dict, cells) -> int:
    key = tuple(sorted(r * o.N + c for r, c in cells))
    return cells_of_id[key]


def replay(o: Oracle, name: str):
    with open(os.path.join(GOLDEN, f"gif_{name}.json"), encoding="utf-8") as f:
        game = json.load(f)
    cells = o.action_cells()
    cells_of_id = {tuple(sorted(int(x) for x in row if x >= 0)): i for i, row in enumerate(cells)}
    st = o.init_state()
    counts = []
    for mv in game["placements"]:
        colour = mv["colour"] - 1
        assert Oracle.to_move(st) == colour, "turn order / skip rule disagrees with the recording"
        assert o.game_ended(st) is None
        ids = o.legal_ids(st)
        counts.append(len(ids))
        a = _find_action(o, cells_of_id, mv["cells"])
        assert a in set(ids.tolist())
        st, _ = o.next_state(st, a)
    scores = o.game_ended(st)
    assert scores is not None, "recording ends with nobody able to move"
    assert o.square_counts(st).tolist() == game["final_squares"]
    return st, scores, counts


def test_replay_arena20():
    o = Oracle(20, 4, 5)
    st, scores, counts = replay(o, "arena20")
    assert counts == ARENA_COUNTS
    assert scores.tolist() == [1.0, -1.0, 1.0, -1.0]  # c1/c3 tie at 64 squares


def test_replay_7x7():
    o = Oracle(7, 2, 5)
    _, s_win, _ = replay(o, "win7")
    assert s_win.tolist() == [3.0, -1.0]
    _, s_draw, _ = replay(o, "draw7")
    assert s_draw.tolist() == [1.0, 1.0]


def test_next_state_is_functional(oracle20):
    st = oracle20.init_state()
    before = st.copy()
    ids = oracle20.legal_ids(st)
    oracle20.next_state(st, int(ids[0]))
    assert (st == before).all()
    with pytest.raises(KeyError):
        oracle20.next_state(st, 30432 if 30432 not in set(ids.tolist()) else 0)
