"""Golden vectors for the training loss from the reference's own compute_loss.

Run here (never on the GPU box): `python tests/golden/make_loss_golden.py`.
Loads /root/reference/blokus_rl/neural_network.py by file path (stubs as make_net_golden.py) and
calls BlokusNNetWrapper.compute_loss (neural_network.py:138-157) exactly as train_step does
(neural_network.py:52-85 with the collate of alphazero/dataset.py:50-54: bool masks [B, A],
pi padded to the batch's longest K with pad_sequence, z [B, P]); autograd gives the gradients
w.r.t. the policy output and the value output.

Inputs are regenerable from seeds, so only small arrays are stored:
  logits[b] = default_rng(seed_b).standard_normal(A) * 3 (f32) — any real row works: the
  reference re-normalises over the legal subset; legal ids from oracle random boards; pi a
  seeded Dirichlet over the K legal ids (one row rescaled so sum(pi) != 1, one row with K = 1,
  one with K = 0 in the 7x7 case). Output: tests/golden/loss_golden.npz.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)


def logits_row(seed: int, A: int) -> np.ndarray:
    return (np.random.default_rng(seed).standard_normal(A) * 3).astype(np.float32)


def make_case(oracle, boards, seeds, P, special: bool):
    A = oracle.A
    ids = [np.asarray(oracle.legal_ids(b), dtype=np.int64) for b in boards]
    if special:
        ids[1] = ids[1][:1]        # K = 1
        ids[2] = ids[2][:0]        # K = 0 (no legal move)
    pis = []
    for i, li in enumerate(ids):
        rng = np.random.default_rng(1000 + seeds[i])
        p = rng.dirichlet(np.ones(len(li))).astype(np.float32) if len(li) else np.zeros(0, np.float32)
        if special and i == 3:
            p = (p * 0.7).astype(np.float32)
        pis.append(p)
    rng = np.random.default_rng(77 + len(boards))
    v_pred = rng.uniform(-1, 1, (len(boards), P)).astype(np.float32)
    v_gt = rng.choice(np.array([-1.0, 1.0, 3.0], np.float32), (len(boards), P)).astype(np.float32)
    return A, ids, pis, v_pred, v_gt


def reference_loss(nw, A, ids, pis, v_pred, v_gt, seeds):
    from torch.nn.utils.rnn import pad_sequence

    B = len(ids)
    logits = torch.from_numpy(np.stack([logits_row(s, A) for s in seeds])).requires_grad_(True)
    vp = torch.from_numpy(v_pred).requires_grad_(True)
    masks = torch.zeros((B, A), dtype=torch.bool)
    for b, li in enumerate(ids):
        masks[b, torch.from_numpy(li)] = True
    p_gt = pad_sequence([torch.from_numpy(p) for p in pis], batch_first=True)
    w = nw.BlokusNNetWrapper.__new__(nw.BlokusNNetWrapper)  # compute_loss only needs get_valid_dist
    loss = w.compute_loss(masks, (logits, vp), (p_gt, torch.from_numpy(v_gt)))
    loss.backward()
    g = logits.grad.numpy()
    off = g.copy()
    for b, li in enumerate(ids):
        off[b, li] = 0
    assert np.abs(off).max() == 0.0  # the reference gradient lives on the legal ids only
    gsparse = np.concatenate([g[b, li] for b, li in enumerate(ids)]) if B else np.zeros(0)
    return float(loss.item()), gsparse.astype(np.float32), vp.grad.numpy().astype(np.float32)


def main():
    from make_net_golden import load_reference
    from oracle.oracle import Oracle

    torch.set_num_threads(4)
    _, nw = load_reference()
    out = {}
    for tag, (n, P, plies, nb, special) in {"c7": (7, 2, 10, 6, True), "c20": (20, 4, 24, 5, False)}.items():
        o = Oracle(n, P, 5)
        seeds = [31 * (i + 1) + n for i in range(nb)]
        boards = [o.random_board(s, plies) for s in seeds]
        A, ids, pis, v_pred, v_gt = make_case(o, boards, seeds, P, special)
        loss, gsp, gv = reference_loss(nw, A, ids, pis, v_pred, v_gt, seeds)
        out[f"{tag}_A"] = np.int64(A)
        out[f"{tag}_seeds"] = np.asarray(seeds, np.int64)
        out[f"{tag}_k"] = np.asarray([len(x) for x in ids], np.int64)
        out[f"{tag}_ids"] = np.concatenate(ids).astype(np.int32)
        out[f"{tag}_pi"] = np.concatenate(pis).astype(np.float32)
        out[f"{tag}_v_pred"] = v_pred
        out[f"{tag}_v_gt"] = v_gt
        out[f"{tag}_loss"] = np.float64(loss)
        out[f"{tag}_grad_p"] = gsp
        out[f"{tag}_grad_v"] = gv
        print(tag, "A", A, "K", out[f"{tag}_k"].tolist(), "loss", loss)
    fp = os.path.join(HERE, "loss_golden.npz")
    np.savez_compressed(fp, **out)
    print(fp, os.path.getsize(fp), "bytes")


if __name__ == "__main__":
    main()
