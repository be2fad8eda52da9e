"""Replay on disk.

* Packed binary shards — the rows of blokus_rl_amd/replay.py written as they sit in HBM:
  a 64-byte header then `rows x stride` bytes. Readers memory-map the file and copy it to the
  device in one transfer; no per-example Python objects. Header (little endian):
      magic  b"BKREPLAY"  | version u32 = 1 | N u32 | P u32 | cap u32 | stride u32 | pad u32 |
      rows u64 | iteration i64 | reserved (16 B, zero)
  Directory layout mirrors the reference's data/train/iteration_<i>/ (trainer.py:151-154):
      <data_dir>/iteration_<i>/shard_<rank>.bkrp
* The legacy layout — the reference's pickled list of [obs f32/uint8 [2P,N,N], mask f64 [A],
  pi f32 [K], z f64 [P]] per example in iteration_<i>/checkpoint_<e>.examples
  (trainer.py:287-292, dataset.py:29-36) — with a writer (from packed rows) and a reader (to
  packed rows). The reader unpickles through an allow-list (numpy arrays, dtypes, lists), never
  arbitrary callables. A legacy example carries no piece inventory, so its packed state keeps
  the occupancy + player to move (all the observation needs), pieces = 0, flag bit 8 set.
"""
from __future__ import annotations

import io
import pickle
import struct
from pathlib import Path

import numpy as np
import torch

from . import replay as rp

MAGIC = b"BKREPLAY"
VERSION = 1
HEADER_BYTES = 64
_HDR = struct.Struct("<8sIIIIIIQq16s")
assert _HDR.size == HEADER_BYTES
FLAG_LEGACY = 1 << 8

# state word offsets (include/blokus_engine.h)
_W_TO_MOVE, _W_PLY, _W_FLAGS = 86, 87, 88
_MAXN = 20


def write_shard(path, rows: torch.Tensor, cap: int, N: int, P: int, iteration: int = 0) -> Path:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    rows = rows.contiguous()
    E, stride = rows.shape
    if stride != rp.stride_of(cap):
        raise ValueError(f"row stride {stride} != stride_of({cap})")
    host = rows.cpu().numpy()
    with open(path, "wb") as f:
        f.write(_HDR.pack(MAGIC, VERSION, N, P, cap, stride, 0, E, iteration, b"\0" * 16))
        f.write(host.tobytes())
    return path


def read_header(path) -> dict:
    with open(path, "rb") as f:
        raw = f.read(HEADER_BYTES)
    if len(raw) != HEADER_BYTES:
        raise ValueError(f"{path}: truncated header")
    magic, ver, N, P, cap, stride, _, E, it, _ = _HDR.unpack(raw)
    if magic != MAGIC or ver != VERSION:
        raise ValueError(f"{path}: not a packed replay shard (magic {magic!r}, version {ver})")
    if stride != rp.stride_of(cap):
        raise ValueError(f"{path}: stride {stride} does not match cap {cap}")
    return {"N": N, "P": P, "cap": cap, "stride": stride, "rows": E, "iteration": it}


def read_shard(path, device: str | torch.device = "cpu") -> tuple[torch.Tensor, dict]:
    """-> (rows uint8 [E, stride] on `device`, header)."""
    h = read_header(path)
    mm = np.memmap(path, dtype=np.uint8, mode="r", offset=HEADER_BYTES, shape=(h["rows"], h["stride"]))
    rows = torch.from_numpy(np.array(mm)).to(device)
    return rows, h


def shard_path(data_dir, iteration: int, rank: int = 0) -> Path:
    return Path(data_dir) / f"iteration_{iteration}" / f"shard_{rank}.bkrp"


def list_shards(data_dir, last_iterations: int | None = None) -> list[Path]:
    """Shards of the last `last_iterations` iterations (the reference's history window)."""
    its = sorted((int(p.name.split("_")[1]), p) for p in Path(data_dir).glob("iteration_*") if p.is_dir())
    if last_iterations is not None:
        its = its[-last_iterations:]
    return [s for _, d in its for s in sorted(d.glob("shard_*.bkrp"))]


# ----------------------------------------------------------------------------- legacy layout
class _AllowListUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"), ("builtins", "list"), ("builtins", "tuple"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"legacy replay: refusing to load {module}.{name}")


def load_legacy(path) -> list:
    with open(path, "rb") as f:
        return _AllowListUnpickler(io.BytesIO(f.read())).load()


def save_legacy(path, examples: list):
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    with open(path, "wb+") as f:
        pickle.Pickler(f).dump(examples)


def packed_to_legacy(rows: torch.Tensor, cap: int, engine) -> list:
    """Packed rows -> reference examples [obs f32 [2P,N,N], mask f64 [A], pi f32 [K], z f64 [P]];
    obs via bk_observe, the mask is the row's legal-id list."""
    u = rp.unpack(rows.to(engine.device), cap, engine.P)
    obs = engine.observe(u["states"].contiguous()).cpu().numpy()
    k = u["k"].cpu().numpy()
    ids = u["ids"].cpu().numpy().astype(np.int64)
    pi = u["pi"].cpu().numpy()
    z = u["z"].cpu().numpy().astype(np.float64)
    out = []
    for i in range(rows.shape[0]):
        mask = np.zeros(engine.A, dtype=np.float64)
        mask[ids[i, : k[i]]] = 1.0
        out.append([obs[i], mask, pi[i, : k[i]].copy(), z[i]])
    return out


def legacy_to_packed(examples: list, N: int, P: int, cap: int | None = None) -> tuple[torch.Tensor, int]:
    """Reference examples -> packed rows (CPU tensor). The state keeps occupancy (planes 0..P-1)
    and the player to move (the one-hot plane among P..2P-1)."""
    E = len(examples)
    ks = [int(np.count_nonzero(np.asarray(ex[1]))) for ex in examples]
    if cap is None:
        cap = max(64, (max(ks, default=1) + 63) // 64 * 64)
    states = np.zeros((E, rp.STATE), dtype=np.uint8)
    words = states.view(np.uint32)
    ids = np.full((E, cap), -1, dtype=np.int32)
    pi = np.zeros((E, cap), dtype=np.float32)
    z = np.zeros((E, P), dtype=np.float32)
    k = np.asarray(ks, dtype=np.int32)
    bit = (np.uint32(1) << np.arange(N, dtype=np.uint32))
    for i, ex in enumerate(examples):
        obs = np.asarray(ex[0])
        if obs.shape != (2 * P, N, N):
            raise ValueError(f"example {i}: observation shape {obs.shape} != {(2 * P, N, N)}")
        occ = (obs[:P] != 0)
        words[i, : P * _MAXN].reshape(P, _MAXN)[:, :N] = (occ * bit).sum(axis=2, dtype=np.uint64).astype(np.uint32)
        tm = np.flatnonzero(obs[P:].reshape(P, -1).any(axis=1))
        words[i, _W_TO_MOVE] = int(tm[0]) if len(tm) else 0
        words[i, _W_PLY] = int(occ.sum())  # squares placed (the ply count is not recoverable)
        words[i, _W_FLAGS] = FLAG_LEGACY
        li = np.flatnonzero(np.asarray(ex[1]))
        if len(li) > cap:
            raise ValueError(f"example {i}: K={len(li)} > cap {cap}")
        ids[i, : len(li)] = li
        p = np.asarray(ex[2], dtype=np.float32).reshape(-1)
        pi[i, : len(p)] = p[: cap]
        z[i] = np.asarray(ex[3], dtype=np.float32).reshape(-1)[:P]
    buf, cap = rp.pack(torch.from_numpy(states), torch.from_numpy(ids), torch.from_numpy(pi), torch.from_numpy(k),
                       torch.from_numpy(z), cap=cap)
    return buf, cap
