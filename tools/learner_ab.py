"""Learner step A/B (§8f row 1): ms per Adam step at batch B of the 20x20 ResNet-5x64 under
framework-level choices — MIOpen vs native batch norm, NCHW vs channels_last, MIOpen find mode, the tower convs on bk_conv_x3 ("x3": Learner(device_path=True)) —
on the same device replay batches. Prints one JSON line per configuration.

    python tools/learner_ab.py [--batch 1024] [--steps 20] [--configs base,nativebn,...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from blokus_rl_amd.alphazero.learner import DeviceReplay, Learner  # noqa: E402
from blokus_rl_amd.alphazero.learner_bench import synthetic_replay  # noqa: E402
from blokus_rl_amd.engine import Engine  # noqa: E402
from blokus_rl_amd.nets import ResNet, use_native_batchnorm  # noqa: E402


def run(cfg: str, eng, rb, rows: int, batch: int, steps: int) -> dict:
    torch.backends.cudnn.benchmark = "bench" in cfg
    torch.manual_seed(0)
    model = ResNet(eng.N, eng.P, eng.A, 5).to(eng.device)
    if "nativebn" in cfg:
        use_native_batchnorm(model)
    cl = "cl" in cfg.split("+")
    if cl:
        model = model.to(memory_format=torch.channels_last)
    L = Learner(model, lr=1e-3, weight_decay=1e-4, batch_size=batch, seed=0, device_path="x3" in cfg)
    cl = cl or "x3" in cfg
    gen = torch.Generator(device=eng.device).manual_seed(0)
    idx = [torch.randint(0, rows, (batch,), device=eng.device, generator=gen) for _ in range(steps + 5)]

    def batch_of(i):
        b = rb.batch(idx[i])
        if cl:
            b["observation"] = b["observation"].contiguous(memory_format=torch.channels_last)
        return b

    for i in range(5):
        L.train_step(batch_of(i))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(5, 5 + steps):
        loss = L.train_step(batch_of(i))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"config": cfg, "batch": batch, "ms_per_step": dt / steps * 1e3, "samples_per_s": batch * steps / dt,
            "loss": float(loss)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--configs", default="base,cl+nativebn,x3")
    a = ap.parse_args()
    eng = Engine(20, 4, 5)
    buf, cap, *_ = synthetic_replay(eng, a.rows, seed=0)
    rb = DeviceReplay(eng, cap=cap)
    rb.add_packed(buf, cap)
    for rnd in range(2):
        for cfg in a.configs.split(","):
            r = run(cfg, eng, rb, a.rows, a.batch, a.steps)
            r["round"] = rnd
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
