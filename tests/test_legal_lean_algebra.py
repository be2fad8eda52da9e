"""Host check of the lean legal-mask step's algebra (legal_rows.h, orient_step SPLIT 3: the default
k_legal_mask_rows and its multi-wave variants) against the oracle, before any GPU run: the lane arithmetic of one origin row — forbidden rows with the columns >= N and the rows past the board set (no column or
row masks), the field's bit offset as base + rw[w], the 64-bit shift split over two words — is
restated in 32-bit Python integers and must give the oracle's masks bit for bit
(blokus_wrapper.py:108-132 via the oracle, oracle/oracle.py)."""
import os
import re

import numpy as np
import pytest

from oracle.oracle import Oracle

HERE = os.path.dirname(os.path.abspath(__file__))
M32 = 0xFFFFFFFF


def _orient_table():
    src = open(os.path.join(HERE, "..", "blokus_rl_amd", "csrc", "orient_table.h")).read()
    rows = re.findall(r"\{(\d+), (\d+), (\d+), (\d+), \{([\d, ]+)\}, \{([\d, ]+)\}\}", src)
    out = []
    for p, h, w, n, dr, dc in rows:
        n = int(n)
        out.append((int(p), int(h), int(w), [int(x) for x in dr.split(",")][:n],
                    [int(x) for x in dc.split(",")][:n]))
    assert len(out) == 91
    return out


def _corners(N: int, P: int):
    if P == 4:
        return [(0, 0), (0, N - 1), (N - 1, 0), (N - 1, N - 1)]
    return [(0, 0), (N - 1, N - 1)]


def _lean_mask(st: np.ndarray, N: int, P: int, num_pieces: int, rng) -> np.ndarray:
    words = st.view(np.uint32)
    q = int(words[86])
    full = (1 << N) - 1
    own = [int(words[q * 20 + r]) for r in range(N)]
    occ = [int(words[r] | words[20 + r] | words[40 + r] | words[60 + r]) for r in range(N)]
    pieces = int(words[80 + q])
    first = not any(own)
    cr, cc = _corners(N, P)[q]
    forb, anch = [], []
    for r in range(N):
        up = own[r - 1] if r > 0 else 0
        dn = own[r + 1] if r + 1 < N else 0
        forb.append((occ[r] | own[r] << 1 | own[r] >> 1 | up | dn) & full)
        if first:
            anch.append((1 << cc) if r == cr else 0)
        else:
            anch.append((up << 1 | up >> 1 | dn << 1 | dn >> 1) & full)
    table = _orient_table()
    nbits = sum((N - h + 1) * (N - w + 1) for p, h, w, _, _ in table if p < num_pieces)
    m32 = [0] * ((nbits + 31) // 32 + 2)
    for r in range(N):
        # the lane's five rows: past the board they are another board's rows (random here) for the
        # anchors, and all-forbidden for fr
        fr, ar = [], []
        for d in range(5):
            if r + d < N:
                f, a = forb[r + d] | (~full & M32), anch[r + d]
            else:
                f, a = M32, int(rng.integers(0, 1 << 32))
            fr.append(f)
            ar.append(a)
        rN1 = r * (N + 1)
        base = 0
        for p, h, w, dr, dc in table:
            if p >= num_pieces:
                continue
            bad = good = 0
            for a, b in zip(dr, dc):  # cell (dr, dc) of origin column c: bit c of row[dr] >> dc
                bad |= fr[a] >> b
                good |= ar[a] >> b
            pm = M32 if (pieces >> p) & 1 else 0
            v = good & ~bad & pm & M32
            bit = base + rN1 - r * w
            x = v << (bit & 31)
            m32[bit >> 5] |= x & M32
            m32[(bit >> 5) + 1] |= x >> 32
            base += (N - h + 1) * (N - w + 1)
    return np.array(m32, dtype=np.uint64)


@pytest.mark.parametrize("preset,nboards", [((20, 4, 5), 6), ((7, 2, 5), 8), ((7, 2, 4), 8)])
def test_lean_step_algebra_matches_oracle(preset, nboards):
    o = Oracle(*preset)
    rng = np.random.default_rng(11)
    for k in range(nboards):
        st = o.random_board(seed=100 + k, max_plies=6 * preset[1] + 4 * k)
        mask, _ = o.legal_mask(st)
        ref32 = mask.view(np.uint32).astype(np.uint64)
        got = _lean_mask(st, preset[0], preset[1], o.num_pieces, rng)
        assert (got[: len(ref32)] == ref32).all(), (preset, k)
        assert not got[len(ref32):].any()
