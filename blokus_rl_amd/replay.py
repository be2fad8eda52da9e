"""Packed replay examples and their cross-GPU exchange.

One example = fixed-stride bytes:  state (384) | k int32 | player int32 | z f32[4] |
ids int16[cap] | pi f32[cap]   (cap = the batch's largest K rounded up to 64; the legal-move
mask and observation are NOT sent: the receiver recomputes them with bk_legal_mask /
bk_observe). Self-play ranks own disjoint games; the only collective of the path is one
all_gather of these rows per iteration, over RCCL (xGMI) on GPUs or gloo on CPU.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

STATE = 384
HEADER = STATE + 4 + 4 + 16


def dist_active() -> bool:
    """A process group is up (also at world size 1: `BK_DIST_BACKEND=nccl python bench.py --gpus 1`
    runs the collectives of the multi-GPU path on one device)."""
    return dist.is_available() and dist.is_initialized()


def stride_of(cap: int) -> int:
    s = HEADER + cap * 2 + cap * 4
    return (s + 15) // 16 * 16


def pack(states: torch.Tensor, ids: torch.Tensor, pi: torch.Tensor, k: torch.Tensor, z: torch.Tensor,
         player: torch.Tensor | None = None, cap: int | None = None) -> tuple[torch.Tensor, int]:
    """-> (uint8 [E, stride], cap)."""
    E = states.shape[0]
    if cap is None:
        kmax = int(k.max().item()) if E else 1
        cap = max(64, (kmax + 63) // 64 * 64)
    dev = states.device
    out = torch.zeros((E, stride_of(cap)), dtype=torch.uint8, device=dev)
    out[:, :STATE] = states
    out[:, STATE:STATE + 4] = k.to(torch.int32).contiguous().view(torch.uint8).view(E, 4)
    pl = player if player is not None else torch.full((E,), -1, dtype=torch.int32, device=dev)
    out[:, STATE + 4:STATE + 8] = pl.to(torch.int32).contiguous().view(torch.uint8).view(E, 4)
    zz = torch.zeros((E, 4), dtype=torch.float32, device=dev)
    zz[:, : z.shape[1]] = z.float()
    out[:, STATE + 8:HEADER] = zz.contiguous().view(torch.uint8).view(E, 16)
    w = min(cap, ids.shape[1])
    idc = torch.full((E, cap), -1, dtype=torch.int16, device=dev)
    idc[:, :w] = ids[:, :w].to(torch.int16)
    pic = torch.zeros((E, cap), dtype=torch.float32, device=dev)
    pic[:, :w] = pi[:, :w].float()
    out[:, HEADER:HEADER + 2 * cap] = idc.view(torch.uint8).view(E, 2 * cap)
    out[:, HEADER + 2 * cap:HEADER + 6 * cap] = pic.view(torch.uint8).view(E, 4 * cap)
    return out, cap


def unpack(buf: torch.Tensor, cap: int, P: int = 4) -> dict:
    E = buf.shape[0]
    b = buf.contiguous()
    return {
        "states": b[:, :STATE].clone(),
        "k": b[:, STATE:STATE + 4].clone().view(torch.int32).view(E),
        "player": b[:, STATE + 4:STATE + 8].clone().view(torch.int32).view(E),
        "z": b[:, STATE + 8:HEADER].clone().view(torch.float32).view(E, 4)[:, :P],
        "ids": b[:, HEADER:HEADER + 2 * cap].clone().view(torch.int16).view(E, cap),
        "pi": b[:, HEADER + 2 * cap:HEADER + 6 * cap].clone().view(torch.float32).view(E, cap),
    }


def all_gather_packed(buf: torch.Tensor, cap: int, group=None) -> tuple[torch.Tensor, int]:
    """Gather every rank's packed rows (ragged row counts and caps) -> (rows of all ranks in rank
    order, common cap). Rows are re-packed to the largest cap first so one fixed-stride
    collective moves them: all_gather_into_tensor on RCCL, all_gather on gloo."""
    world = dist.get_world_size(group)
    dev = buf.device
    meta = torch.tensor([buf.shape[0], cap], dtype=torch.int64, device=dev)
    metas = [torch.zeros_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    counts = [int(m[0]) for m in metas]
    cmax = max(int(m[1]) for m in metas)
    if cmax != cap:
        u = unpack(buf, cap)
        buf, cap = pack(u["states"], u["ids"], u["pi"], u["k"], u["z"], u["player"], cap=cmax)
    emax = max(counts)
    stride = stride_of(cmax)
    padded = torch.zeros((emax, stride), dtype=torch.uint8, device=dev)
    padded[: buf.shape[0]] = buf
    if dist.get_backend(group) == "nccl":
        gathered = torch.empty((world * emax, stride), dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(gathered, padded, group=group)
        parts = gathered.view(world, emax, stride)
        rows = [parts[r, : counts[r]] for r in range(world)]
    else:
        parts = [torch.empty_like(padded) for _ in range(world)]
        dist.all_gather(parts, padded, group=group)
        rows = [parts[r][: counts[r]] for r in range(world)]
    return torch.cat(rows), cmax
