"""Replay on disk: packed binary shards and the reference's pickled
example layout (trainer.py:287-292, dataset.py:29-54), both directions."""
import collections
import pickle

import numpy as np
import pytest
import torch

from oracle.oracle import Oracle


def _random_rows(E, seed, cap=128, P=4):
    from blokus_rl_amd import replay as rp

    g = torch.Generator().manual_seed(seed)
    states = torch.randint(0, 256, (E, 384), dtype=torch.uint8, generator=g)
    k = torch.randint(0, cap, (E,), dtype=torch.int32, generator=g)
    ids = torch.randint(0, 30433, (E, cap), dtype=torch.int32, generator=g)
    pi = torch.rand((E, cap), generator=g)
    z = torch.randn((E, P), generator=g)
    return rp.pack(states, ids, pi, k, z, cap=cap)


def test_shard_round_trip(tmp_path):
    from blokus_rl_amd import replay_io as rio

    rows, cap = _random_rows(37, 0)
    p = rio.write_shard(rio.shard_path(tmp_path, 3, 1), rows, cap, 20, 4, iteration=3)
    h = rio.read_header(p)
    assert h == {"N": 20, "P": 4, "cap": cap, "stride": rows.shape[1], "rows": 37, "iteration": 3}
    back, _ = rio.read_shard(p)
    assert torch.equal(back, rows)
    assert p.stat().st_size == rio.HEADER_BYTES + rows.numel()


def test_shard_window_and_bad_files(tmp_path):
    from blokus_rl_amd import replay_io as rio

    for it in (1, 2, 3, 10):
        rows, cap = _random_rows(4, it)
        rio.write_shard(rio.shard_path(tmp_path, it, 0), rows, cap, 20, 4, iteration=it)
    names = [p.parent.name for p in rio.list_shards(tmp_path, last_iterations=2)]
    assert names == ["iteration_3", "iteration_10"]
    bad = tmp_path / "bad.bkrp"
    bad.write_bytes(b"NOTREPLY" + b"\0" * 100)
    with pytest.raises(ValueError):
        rio.read_header(bad)


def _legacy_examples(o: Oracle, n, seed):
    rng = np.random.default_rng(seed)
    out, states = [], []
    for i in range(n):
        s = o.random_board(seed * 100 + i, 30)
        ids = o.legal_ids(s)
        if len(ids) == 0:
            continue
        mask = np.zeros(o.A, dtype=np.float64)
        mask[ids] = 1
        pi = rng.dirichlet(np.ones(len(ids))).astype(np.float32)
        z = rng.choice([-1.0, 1.0, 3.0], o.P).astype(np.float64)
        out.append([o.observe(s).astype(np.float32), mask, pi, z])
        states.append(s)
    return out, states


@pytest.mark.parametrize("n,p", [(20, 4), (7, 2)])
def test_legacy_to_packed_keeps_everything_training_reads(n, p):
    from blokus_rl_amd import replay as rp
    from blokus_rl_amd import replay_io as rio

    o = Oracle(n, p, 5)
    ex, states = _legacy_examples(o, 12, 7)
    rows, cap = rio.legacy_to_packed(ex, n, p)
    u = rp.unpack(rows, cap, p)
    for i, (obs, mask, pi, z) in enumerate(ex):
        K = int(mask.sum())
        assert int(u["k"][i]) == K
        assert np.array_equal(u["ids"][i, :K].numpy(), np.flatnonzero(mask))
        assert np.array_equal(u["pi"][i, :K].numpy(), pi)
        assert np.array_equal(u["z"][i].numpy(), z.astype(np.float32))
        w = u["states"][i].numpy().view(np.uint32)
        ref = states[i].view(np.uint32)
        assert np.array_equal(w[: 4 * 20], ref[: 4 * 20])          # occupancy bitboards
        assert w[86] == ref[86] and w[88] == rio.FLAG_LEGACY        # to-move, legacy flag
        assert np.array_equal(o.observe(u["states"][i].numpy()), obs)  # the observation is reproduced


def test_legacy_pickle_round_trip_and_allow_list(tmp_path):
    from blokus_rl_amd import replay_io as rio

    o = Oracle(7, 2, 5)
    ex, _ = _legacy_examples(o, 5, 3)
    fp = tmp_path / "iteration_1" / "checkpoint_0.examples"
    rio.save_legacy(fp, ex)
    back = rio.load_legacy(fp)
    assert len(back) == len(ex)
    for a, b in zip(ex, back):
        for x, y in zip(a, b):
            assert np.array_equal(x, y) and x.dtype == y.dtype
    evil = tmp_path / "evil.examples"
    evil.write_bytes(pickle.dumps(collections.OrderedDict(a=1)))  # a global outside the allow-list
    with pytest.raises(pickle.UnpicklingError):
        rio.load_legacy(evil)


@pytest.mark.gpu
def test_packed_to_legacy_round_trip():
    from blokus_rl_amd import replay_io as rio
    from blokus_rl_amd.engine import Engine

    eng = Engine(20, 4, 5)
    o = Oracle(20, 4, 5)
    ex, _ = _legacy_examples(o, 10, 5)
    rows, cap = rio.legacy_to_packed(ex, 20, 4)
    back = rio.packed_to_legacy(rows, cap, eng)
    for a, b in zip(ex, back):
        assert np.array_equal(a[0], b[0])
        assert np.array_equal(a[1], b[1])
        assert np.array_equal(a[2], b[2])
        assert np.array_equal(a[3], b[3])
