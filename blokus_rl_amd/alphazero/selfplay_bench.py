"""bench.py --workload selfplay: AlphaZero self-play sims/s (BASELINE.json configs 3 and 4).

Per GPU: 256 concurrent 4-player 20x20 games, 100 MCTS simulations per move, cpuct 1,
temperature 1, first-ply Dirichlet(1) x 0.25, ResNet (5 blocks, 64 channels, A=30433,
24.78M params) with random-init weights (seed 0) as the leaf evaluator in fp32. A step = one
ply of every game (= 256 x 100 simulations). Ranks play independent games (seeded by rank).
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

from ..engine import Engine
from ..nets import build_model
from .selfplay import SelfPlay

# Leaf-eval FLOPs of the default ResNet: 347.5 MFLOP per leaf.
RESNET_FLOPS_PER_LEAF = 347.5e6
FP32_PEAK = 157.3e12


def bench_selfplay(args, world, rank):
    torch.manual_seed(0)
    eng = Engine(20, 4, 5)
    G = args.games
    model = build_model(args.model, 20, 4, eng.A, num_res_blocks=5).to(eng.device).eval()
    nn_dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[args.nn_dtype]
    sp = SelfPlay(eng, model, G, num_sims=args.sims, seed=1234 + rank, nn_dtype=nn_dtype,
                  node_cap=args.node_cap, continuous=True)
    for _ in range(args.warmup):
        sp.play_ply()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    sims0 = sp.stats.sims
    sp.enable_timers(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sp.play_ply()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    sims = sp.stats.sims - sims0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        s = torch.tensor([sims], dtype=torch.float64, device="cuda")
        dist.all_reduce(s)
        sims = int(s.item())
    ms = sp.timer_ms()
    counters = sp.mcts.check()
    return {
        "metric": "MCTS sims/sec on 20x20 Blokus (4 players, 256 games/GPU, 100 sims/move)",
        "value": sims / elapsed,
        "unit": "sims/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": f"{args.nn_dtype} net / f64 search / u32 bitboards",
        "data": "synthetic: self-play from the empty board, random-init ResNet weights (seed 0)",
        "config": {"workload": "config 3/4: AlphaZero self-play 20x20, 256 concurrent games per GPU, 100 sims/move",
                   "global_batch": G * world, "parallelism": f"dp{world} (independent games)",
                   "model": args.model},
        "stage_ms_per_sim_step": ms,
        "engine_counters": counters,
        "_selfplay": sp,
    }
