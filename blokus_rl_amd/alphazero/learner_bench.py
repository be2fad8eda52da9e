"""Learner throughput: AlphaZero training samples/s on the device path
(DeviceReplay -> bk_replay_batch -> ResNet fwd/bwd -> bk_policy_loss(+grad) -> Adam, DDP over
RCCL when several ranks run), next to the reference-layout path timed on the same box
(host examples [obs, f64 mask, f32 pi, f64 z] -> pad_sequence collate -> H2D -> per-sample
masked_select/log_softmax loss loop, neural_network.py:52-85/138-157, dataset.py:38-54)."""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.nn.functional as F

from .. import replay as rp
from ..boards import random_boards
from ..engine import _check, _ptr, _stream, load_library
from ..nets import ResNet
from .learner import DeviceReplay, Learner


def synthetic_replay(eng, rows: int, seed: int, cap: int = 1024):
    """`rows` examples of the packed replay layout: random-play 20x20 boards, pi = a seeded
    Dirichlet(1) over each board's legal ids, z = a -1/3/1 outcome row."""
    states = random_boards(eng, rows, seed0=seed, max_plies=60)
    ids, counts = eng.legal_ids(states, cap=cap)
    k = counts.clamp(min=0)
    g = torch.Generator(device=eng.device).manual_seed(seed)
    e = -torch.log(torch.rand(ids.shape, device=eng.device, generator=g).clamp(min=1e-12))
    e = e * (torch.arange(cap, device=eng.device) < k.unsqueeze(1))
    pi = e / e.sum(1, keepdim=True).clamp(min=1e-12)
    win = torch.randint(0, eng.P, (rows,), device=eng.device, generator=g)
    z = torch.full((rows, eng.P), -1.0, device=eng.device)
    z[torch.arange(rows, device=eng.device), win] = 3.0
    buf, c = rp.pack(states, ids, pi, k, z, cap=cap)
    return buf, c, states, ids, pi, k, z


def loss_kernel_bytes(k: torch.Tensor) -> float:
    """Algorithmic bytes of bk_policy_loss + bk_policy_loss_grad for rows with K ids each:
    forward reads K x (id 2 + logit 4 + pi 4) + K count + writes loss/lse (8); the gradient
    reads the same + lse and writes K logits' gradients (4 each)."""
    K = k.double()
    return float(((10 * K + 12) + (10 * K + 8 + 4 * K)).sum())


def time_loss_kernels(x, ids, pi, k, reps: int = 50):
    lib = load_library()
    B = x.shape[0]
    loss = torch.empty(B, device=x.device)
    lse = torch.empty(B, device=x.device)
    grad = torch.zeros_like(x)
    s = _stream(x.device)

    def once():
        _check(lib.bk_policy_loss(_ptr(x), x.shape[1], _ptr(ids), _ptr(pi), _ptr(k), ids.shape[1], B, _ptr(loss),
                                  _ptr(lse), s))
        _check(lib.bk_policy_loss_grad(_ptr(x), x.shape[1], _ptr(ids), _ptr(pi), _ptr(k), ids.shape[1], B, _ptr(lse),
                                       1.0 / B, None, _ptr(grad), grad.shape[1], s))

    for _ in range(5):
        once()
    st = torch.cuda.current_stream(x.device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        once()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def time_conv_x3(batch: int, device, reps: int = 20) -> dict:
    """k_conv_x3 alone at the learner's batch (HIP events on the stream it launches on): its
    executed MFMA work per launch = batch x 4 waves x 25 pixel groups x 18 K-chunks x 3 products
    of v_mfma_f32_16x16x32_f16 (16384 FLOP each); the fp32-equivalent conv = 2 x batch x 400 x 64 x 576."""
    from .train_conv import conv_x3, pack_weight

    g = torch.Generator(device=device).manual_seed(0)
    x = torch.randn(batch, 64, 20, 20, device=device, generator=g).contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, 64, 3, 3, device=device, generator=g) * 0.06
    ws, inv = pack_weight(w, False)
    for _ in range(3):
        conv_x3(x, ws, inv, None)
    st = torch.cuda.current_stream(device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        conv_x3(x, ws, inv, None)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return {"kernel": "k_conv_x3", "ms": ms, "flop": float(batch) * 4 * 25 * 18 * 3 * 16384,
            "fp32_equiv_flop": 2.0 * batch * 400 * 64 * 576}


def time_conv_x3_wgrad(batch: int, device, reps: int = 20) -> dict:
    """bk_conv_x3_wgrad (k_conv_x3_wgrad + its fixed-order reduce) alone at the learner's batch: its
    executed MFMA work per launch = batch x 8 waves x 15 K-chunks (24-wide rows: 480 of 400 pixels)
    x 54 v_mfma_f32_16x16x32_f16; the fp32-equivalent = 2 x batch x 400 x 64 x 576."""
    from .train_conv import conv_x3_wgrad

    g = torch.Generator(device=device).manual_seed(1)
    x = torch.randn(batch, 64, 20, 20, device=device, generator=g).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(batch, 64, 20, 20, device=device, generator=g).contiguous(memory_format=torch.channels_last)
    for _ in range(3):
        conv_x3_wgrad(x, gy)
    st = torch.cuda.current_stream(device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        conv_x3_wgrad(x, gy)
    e1.record(st)
    torch.cuda.synchronize()
    return {"kernel": "k_conv_x3_wgrad + k_conv_x3_wgrad_reduce", "ms": e0.elapsed_time(e1) / reps,
            "flop": float(batch) * 8 * 15 * 54 * 16384, "fp32_equiv_flop": 2.0 * batch * 400 * 64 * 576}


def reference_loop_loss(masks, p_pred, v_pred, p_gt, v_gt):
    """compute_loss as written in neural_network.py:138-157 (per-sample loop)."""
    v_loss = (v_pred.squeeze() - v_gt).pow(2).mean()
    p_loss = 0
    for mask, gt, logits in zip(masks, p_gt, p_pred):
        pred = F.log_softmax(torch.masked_select(logits, mask), dim=-1)
        pred = F.pad(pred, (0, gt.shape[0] - pred.shape[0]), value=0)
        p_loss += -torch.sum(gt * pred)
    p_loss /= masks.size(0)
    return p_loss + v_loss


def bench_reference_path(eng, states, ids, pi, k, z, batch: int, steps: int, model: torch.nn.Module):
    """Host-resident reference-layout examples through the reference's batch path."""
    from torch.nn.utils.rnn import pad_sequence

    n = min(states.shape[0], batch * (steps + 1))
    obs = eng.observe(states[:n]).cpu().numpy()
    masks = eng.unpack_mask(eng.legal_mask(states[:n])[0]).cpu().numpy().astype(np.float64)
    kk = k[:n].cpu().numpy()
    pis = pi[:n].cpu().numpy()
    zz = z[:n].cpu().numpy().astype(np.float64)
    data = [[obs[i], masks[i], pis[i, : kk[i]].copy(), zz[i]] for i in range(n)]
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-4)
    dev = eng.device

    def step(items):
        b = {"observation": torch.stack([torch.from_numpy(x[0]).float() for x in items]),
             "mask": torch.stack([torch.from_numpy(x[1]).bool() for x in items]),
             "prob": pad_sequence([torch.from_numpy(x[2]).float() for x in items], batch_first=True),
             "score": torch.stack([torch.from_numpy(x[3]).float() for x in items])}
        b = {kk_: v.to(dev) for kk_, v in b.items()}
        model.train()
        p, v = model(b["observation"])
        loss = reference_loop_loss(b["mask"], p, v, b["prob"], b["score"])
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss.item()

    step(data[:batch])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(1, steps + 1):
        step(data[i * batch:(i + 1) * batch])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"value": steps * batch / dt, "unit": "samples/s", "batch": batch, "steps": steps,
            "kind": "port", "cores": 1,
            "sample": f"{steps} reference-layout train steps at batch {batch} (host examples, pad collate, "
                      f"H2D, per-sample loss loop; same ResNet on the same GPU) in {dt:.2f} s"}


def bench_learner(eng, world: int, rank: int, batch: int, steps: int, warmup: int, rows: int = 8192,
                  reference_steps: int = 0, barrier=None, device_path: bool | str = "auto"):
    buf, cap, states, ids, pi, k, z = synthetic_replay(eng, rows, seed=1000 * rank)
    rb = DeviceReplay(eng, cap=cap)
    rb.add_packed(buf, cap)
    torch.manual_seed(0)
    model = ResNet(eng.N, eng.P, eng.A, 5).to(eng.device)
    L = Learner(model, lr=1e-3, weight_decay=1e-4, batch_size=batch, seed=rank, device_path=device_path)
    gen = torch.Generator(device=eng.device).manual_seed(rank)
    idx = [torch.randint(0, rows, (batch,), device=eng.device, generator=gen) for _ in range(steps + warmup)]
    for i in range(warmup):
        L.train_step(rb.batch(idx[i]))
    torch.cuda.synchronize()
    if barrier:
        barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        loss = L.train_step(rb.batch(idx[i]))
    torch.cuda.synchronize()
    if barrier:
        barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # the loss kernels alone on one batch of real net outputs
    with torch.no_grad():
        model.eval()
        b = rb.batch(idx[0])
        lp, _ = model(b["observation"])
    kms = time_loss_kernels(lp.contiguous(), b["ids"], b["pi"], b["k"])
    kbytes = loss_kernel_bytes(b["k"])
    out = {"batch_per_gpu": batch, "steps": steps, "elapsed_s": dt, "loss": float(loss), "device_path": L.device_path,
           "loss_kernels": {"kernel": "k_policy_loss + k_policy_loss_grad", "ms": kms,
                            "bytes_per_launch_pair": kbytes, "achieved_GBps": kbytes / (kms * 1e-3) / 1e9}}
    if L.device_path:
        out["conv_kernel"] = time_conv_x3(batch, eng.device)
        out["wgrad_kernel"] = time_conv_x3_wgrad(batch, eng.device)
    if reference_steps and rank == 0 and world == 1:
        ref_model = ResNet(eng.N, eng.P, eng.A, 5).to(eng.device)
        out["reference_path"] = bench_reference_path(eng, states, ids, pi, k, z, batch, reference_steps, ref_model)
    return out
