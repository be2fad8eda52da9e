"""GPU parity of the HIP rules engine against the C oracle (bit-exact: states, masks, counts,
scores, observations), through the C-ABI (blokus_rl_amd.engine -> libblokus_hip.so).

Covers the wrapper's env calls of the hot path: get_valid_moves,
get_next_state (incl. the skip rule), get_game_ended, get_observation, string_representation,
on random self-played games of both presets, the recorded reference games, and the
config-2 benchmark boards."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

PRESETS = [(20, 4, 5), (7, 2, 5), (7, 2, 4)]


@pytest.fixture(scope="module")
def engines():
    from blokus_rl_amd.engine import Engine
    return {p: Engine(*p) for p in PRESETS}


@pytest.fixture(scope="module")
def oracles():
    return {p: Oracle(*p) for p in PRESETS}


def _np(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("preset", PRESETS)
def test_init_states(engines, oracles, preset):
    eng, o = engines[preset], oracles[preset]
    st = _np(eng.init_states(3))
    ref = o.init_state()
    for b in range(3):
        assert (st[b] == ref).all()
    assert eng.A == o.A


@pytest.mark.parametrize("preset", PRESETS)
def test_lockstep_random_games(engines, oracles, preset):
    """B games played to the end with uniform random legal moves; every ply compares the GPU
    engine with the oracle: legal bitmask + count for the mover and for every other colour,
    next state bytes, next player, terminal flag + scores, observation planes."""
    eng, o = engines[preset], oracles[preset]
    B = 24 if preset[0] == 20 else 64
    rngs = [np.random.default_rng(1000 + b) for b in range(B)]
    st_g = eng.init_states(B)
    st_o = [o.init_state() for _ in range(B)]
    for ply in range(100):
        masks, counts = eng.legal_mask(st_g)
        masks_h, counts_h = _np(masks).view(np.uint64), _np(counts)
        ended, scores = eng.game_ended(st_g)
        ended_h, scores_h = _np(ended), _np(scores)
        obs_h = _np(eng.observe(st_g))
        other = torch.tensor([(ply + b) % o.P for b in range(B)], dtype=torch.int32, device=eng.device)
        m2, c2 = eng.legal_mask(st_g, other)
        m2_h, c2_h = _np(m2).view(np.uint64), _np(c2)
        acts = np.full(B, -1, dtype=np.int32)
        for b in range(B):
            ref_mask, ref_n = o.legal_mask(st_o[b])
            assert counts_h[b] == ref_n, (ply, b)
            assert (masks_h[b] == ref_mask).all(), (ply, b)
            ref_mask2, ref_n2 = o.legal_mask(st_o[b], (ply + b) % o.P)
            assert c2_h[b] == ref_n2 and (m2_h[b] == ref_mask2).all()
            ref_scores = o.game_ended(st_o[b])
            assert bool(ended_h[b]) == (ref_scores is not None)
            if ref_scores is not None:
                assert (scores_h[b] == ref_scores).all()
            assert (obs_h[b] == o.observe(st_o[b])).all()
            if ref_scores is None:
                ids = o.legal_ids(st_o[b])
                acts[b] = int(ids[int(rngs[b].integers(len(ids)))])
                st_o[b], _ = o.next_state(st_o[b], int(acts[b]))
        if (acts < 0).all():
            break
        st_g, nxt, status = eng.next_state(st_g, torch.from_numpy(acts).to(eng.device))
        st_h, nxt_h, status_h = _np(st_g), _np(nxt), _np(status)
        assert (status_h == 0).all()
        for b in range(B):
            assert (st_h[b] == st_o[b]).all(), (ply, b)
            assert nxt_h[b] == Oracle.to_move(st_o[b])
    else:
        pytest.fail("games did not end")
    assert (acts < 0).all()


def test_illegal_action_rejected(engines, oracles):
    eng = engines[(20, 4, 5)]
    st = eng.init_states(2)
    # id 0 = monomino at (0,0): legal for colour 0 on the empty board; id 5 (monomino at (0,5)) is not
    out, nxt, status = eng.next_state(st, torch.tensor([0, 5], dtype=torch.int32, device=eng.device))
    assert _np(status).tolist() == [0, 1]
    assert (_np(out[1]) == _np(st[1])).all()
    assert _np(nxt).tolist() == [1, 0]


@pytest.mark.parametrize("name,preset", [("arena20", (20, 4, 5)), ("win7", (7, 2, 5)), ("draw7", (7, 2, 5))])
def test_recorded_games(engines, oracles, name, preset):
    """Replays the reference's recorded games on the GPU engine."""
    eng, o = engines[preset], oracles[preset]
    with open(os.path.join(GOLDEN, f"gif_{name}.json"), encoding="utf-8") as f:
        game = json.load(f)
    cells_of_id = {tuple(sorted(int(x) for x in row if x >= 0)): i for i, row in enumerate(eng.action_cells)}
    st = eng.init_states(1)
    for mv in game["placements"]:
        assert int(eng.to_move(st)[0]) == mv["colour"] - 1
        a = cells_of_id[tuple(sorted(r * o.N + c for r, c in mv["cells"]))]
        mask, _ = eng.legal_mask(st)
        bits = eng.unpack_mask(mask)[0]
        assert bool(bits[a])
        st, _, status = eng.next_state(st, torch.tensor([a], dtype=torch.int32, device=eng.device))
        assert int(status[0]) == 0
    ended, scores = eng.game_ended(st)
    assert int(ended[0]) == 1
    assert _np(eng.square_counts(st))[0].tolist() == game["final_squares"]


def test_legal_ids_match_mask(engines):
    from blokus_rl_amd.boards import random_boards
    eng = engines[(20, 4, 5)]
    st = random_boards(eng, 64, seed0=7)
    masks, counts = eng.legal_mask(st)
    ids, cnt = eng.legal_ids(st, cap=2048)
    bits = eng.unpack_mask(masks)
    for b in range(64):
        k = int(cnt[b])
        assert k == int(counts[b])
        ref = torch.nonzero(bits[b]).view(-1).to(torch.int32)
        assert torch.equal(ids[b, :k], ref)


def test_benchmark_boards_bit_exact(engines, oracles):
    """Config 2 boards: the GPU-generated boards equal the oracle's recipe byte for byte
    (first 48), and the legal masks of all 4096 equal the oracle's."""
    from blokus_rl_amd.boards import random_boards
    eng, o = engines[(20, 4, 5)], oracles[(20, 4, 5)]
    st = random_boards(eng, 4096, seed0=0)
    st_h = _np(st)
    for b in range(48):
        assert (st_h[b] == o.random_board(b)).all(), b
    masks, counts = eng.legal_mask(st)
    ref_masks, ref_counts = o.legal_mask_batch(st_h)
    assert (_np(counts) == ref_counts).all()
    assert (_np(masks).view(np.uint64) == ref_masks).all()


@pytest.mark.parametrize("B", [1, 2, 4, 5, 1022])
def test_legal_mask_ragged_groups(engines, oracles, B):
    """The classic board's lean kernel handles 3 boards per wave: batches that leave 1 or 2 boards
    in the last group (and batches of one group or less) give the oracle's masks and counts, and
    write nothing past the last board."""
    from blokus_rl_amd.boards import random_boards
    eng, o = engines[(20, 4, 5)], oracles[(20, 4, 5)]
    st = random_boards(eng, B, seed0=11)
    masks = torch.full((B + 1, eng.W), -1, dtype=torch.int64, device=eng.device)
    counts = torch.full((B + 1,), -7, dtype=torch.int32, device=eng.device)
    eng.legal_mask_into(st, masks[:B], counts[:B])
    ref_masks, ref_counts = o.legal_mask_batch(_np(st))
    assert (_np(counts[:B]) == ref_counts).all()
    assert (_np(masks[:B]).view(np.uint64) == ref_masks).all()
    assert int(counts[B]) == -7 and bool((masks[B] == -1).all())


def test_hash_is_board_only(engines, oracles):
    eng, o = engines[(20, 4, 5)], oracles[(20, 4, 5)]
    from blokus_rl_amd.boards import random_boards
    st = _np(random_boards(eng, 32, seed0=3))
    for b in range(32):
        assert int(st[b, 336:344].view(np.uint64)[0]) == o.hash(st[b])


@pytest.mark.parametrize("wpb", ["2", "4", "8", "11", "14", "21", "31", "40", "45", "46", "items"])
def test_legal_kernel_variants_bit_exact(oracles, monkeypatch, wpb):
    """Every k_legal_mask_rows variant (BK_LEGAL_WPB: waves per board group, each wave only its own
    orientations; 11/14 = even and odd origin rows in separate LDS atomics; 21 = two boards per
    wave; 31 = the staged kernel without LDS atomics; 40 = round 4's default step on bit-reversed
    rows; 45 / 46 = the lean step on 3 / 2 waves per group; the default, the lean step on one wave,
    is every other test's) and the item-loop kernel give the oracle's masks on the config-2 boards
    and on 7x7 mid-game boards."""
    from blokus_rl_amd.boards import random_boards
    from blokus_rl_amd.engine import Engine
    if wpb == "items":
        monkeypatch.setenv("BK_LEGAL_KERNEL", "items")
    else:
        monkeypatch.setenv("BK_LEGAL_WPB", wpb)
    for preset, B in (((20, 4, 5), 1024), ((7, 2, 5), 257), ((7, 2, 4), 100)):
        eng, o = Engine(*preset), oracles[preset]
        st = random_boards(eng, B, seed0=5)
        masks, counts = eng.legal_mask(st)
        ref_masks, ref_counts = o.legal_mask_batch(_np(st))
        assert (_np(counts) == ref_counts).all(), preset
        assert (_np(masks).view(np.uint64) == ref_masks).all(), preset
