"""Benchmark of the Blokus hot path on MI355X (contract: one JSON line from rank 0).

Workloads (BASELINE.json configs):
  legal    — config 2: legal-move bitmasks of 4096 random 20x20 boards per step (one
             k_legal_mask launch over the batch), metric = boards/s.
  selfplay — config 3/4: AlphaZero self-play, 256 concurrent 4-player 20x20 games per GPU,
             100 MCTS simulations per move, ResNet leaf evaluation; metric = MCTS sims/s.

Multi-GPU: one process per GPU (torchrun); every rank runs its own independent shard (boards /
games seeded by rank), no data-path collective; value = units of all ranks / max-over-ranks time.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from blokus_rl_amd.replay import dist_active  # noqa: E402

HBM_PEAK = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md chip table)
MFMA_F16_PEAK = 2.5e15  # FLOP/s, dense f16 MFMA (MI355X_MICROARCH.md; not the 2:1-sparsity figure)
MFMA_F32_PEAK = 157.3e12  # FLOP/s, f32-input MFMA = the f32 vector peak (MI355X_MICROARCH.md chip table)

# Algorithmic bytes of one board in k_legal_mask: the packed state read (384 B) + the
# 30433-bit mask written (476 u64 = 3808 B) + its count (4 B). DESIGN.md §4.
LEGAL_BYTES_PER_BOARD = 384 + 3808 + 4


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv: list[str]) -> int:
    """`bench.py --gpus N` started as one process: start N rank processes of this same script
    (torch.distributed.run, one rank per GPU, rendezvous on 127.0.0.1) as CHILD processes and
    return their exit code. Called before anything touches the GPU (this process never
    initialises HIP). Rank 0 prints the one JSON line; the children inherit stdout."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool (RCCL)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env, check=False).returncode


def dist_backend() -> str:
    """RCCL ("nccl") on GPUs; gloo on CPU or when BK_DIST_BACKEND=gloo (several ranks sharing
    one GPU in a rehearsal: RCCL refuses two ranks on one device)."""
    b = os.environ.get("BK_DIST_BACKEND")
    if b:
        return b
    return "nccl" if torch.cuda.is_available() else "gloo"


def _dist_init(need_gpu: bool = True):
    """One process per GPU (torchrun's RANK / LOCAL_RANK / WORLD_SIZE). A process group is made at
    world size > 1, and at world size 1 when BK_DIST_BACKEND is set (e.g. nccl: the multi-GPU
    path's collectives — the all-gather inside the timed region, max-over-ranks timing, DDP — run
    through RCCL on a one-GPU box)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and os.environ.get("BK_DIST_BACKEND"):
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if need_gpu:
        ndev = torch.cuda.device_count()
        if ndev == 0:
            raise RuntimeError("bench.py: no HIP device visible (the workloads run on the GPU; "
                               "--workload dry rehearses the launch on CPU)")
        dev = local % ndev  # one rank per GPU; a gloo rehearsal may put several ranks on one
        torch.cuda.set_device(dev)
    if world > 1 or os.environ.get("BK_DIST_BACKEND"):
        backend = dist_backend() if need_gpu else "gloo"
        kw = {"device_id": torch.device("cuda", torch.cuda.current_device())} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return world, rank, local


def _barrier(world):
    if dist_active():
        dist.barrier()


def _coll_device():
    return "cuda" if dist.get_backend() == "nccl" else "cpu"


def _max_over_ranks(x: float, world: int) -> float:
    if not dist_active():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _sum_over_ranks(x: float, world: int) -> float:
    if not dist_active():
        return x
    t = torch.tensor([float(x)], dtype=torch.float64, device=_coll_device())
    dist.all_reduce(t)
    return float(t.item())


def _dry_rows(rank: int):
    """Rank r's synthetic replay shard for --workload dry: 3 + r rows (ragged across ranks),
    K = 40 + 10 r ids each (so the caps differ: 64 for ranks 0-2, 128 above), seeded by rank."""
    from blokus_rl_amd import replay as rp

    g = torch.Generator().manual_seed(rank)
    E, K = 3 + rank, 40 + 10 * rank
    states = torch.randint(0, 256, (E, rp.STATE), dtype=torch.uint8, generator=g)
    states[:, 0] = rank
    k = torch.randint(1, K + 1, (E,), generator=g).to(torch.int32)
    col = torch.arange(K).unsqueeze(0)
    ids = torch.where(col < k.unsqueeze(1), torch.randint(0, 30433, (E, K), generator=g).to(torch.int16),
                      torch.full((E, K), -1, dtype=torch.int16))
    pi = torch.where(col < k.unsqueeze(1), torch.rand((E, K), generator=g), torch.zeros((E, K)))
    z = torch.tensor([[3.0, -1.0, 1.0, -1.0]]).roll(rank, 1).repeat(E, 1)
    player = (torch.arange(E, dtype=torch.int32) + rank) % 4
    return states, ids, pi, k, z, player


def bench_dry(args, world, rank):
    """--workload dry: the multi-rank launch rehearsed on CPU (gloo, no GPU touched): every rank
    packs a shard of synthetic replay rows (seeded by rank, ragged row counts and caps) and the
    ranks run the config-4 exchange, all_gather_packed; rank 0 checks every rank's rows against
    their generator, field by field (`rows_intact`), and reports which ranks' rows arrived."""
    from blokus_rl_amd import replay as rp

    states, ids, pi, k, z, player = _dry_rows(rank)
    buf, cap = rp.pack(states, ids, pi, k, z, player)
    _barrier(world)
    t0 = time.perf_counter()
    if dist_active():
        rows, cap = rp.all_gather_packed(buf, cap)
    else:
        rows = buf
    _barrier(world)
    dt = _max_over_ranks(time.perf_counter() - t0, world)
    u = rp.unpack(rows, cap)
    seen = sorted({int(s) for s in u["states"][:, 0].tolist()})
    intact, off = True, 0
    for r in range(world):
        st_r, ids_r, pi_r, k_r, z_r, pl_r = _dry_rows(r)
        E, K = ids_r.shape
        sl = slice(off, off + E)
        intact &= (torch.equal(u["states"][sl], st_r) and torch.equal(u["k"][sl], k_r)
                   and torch.equal(u["player"][sl], pl_r) and torch.equal(u["z"][sl], z_r)
                   and torch.equal(u["ids"][sl, :K], ids_r) and torch.equal(u["pi"][sl, :K], pi_r)
                   and bool((u["ids"][sl, K:] == -1).all()) and bool((u["pi"][sl, K:] == 0).all()))
        off += E
    intact &= off == rows.shape[0]
    return {"metric": "launch rehearsal (gloo, CPU): replay rows all-gathered", "value": float(rows.shape[0]),
            "unit": "rows", "n_gpus": world, "steps": 1, "warmup": 0, "ms_per_step": dt * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "dry", "parallelism": f"dp{world}"}, "ranks_seen": seen,
            "rows_intact": bool(intact), "common_cap": cap,
            "backend": dist.get_backend() if dist_active() else None}


def _trace_avg_ms(csv_name: str, kernel_prefix: str):
    """Average duration (ms) of the kernels named kernel_prefix* in a committed rocprofv3
    --kernel-trace --stats summary (profiles/<csv_name>), or None."""
    import csv

    fp = os.path.join(ROOT, "profiles", csv_name)
    if not os.path.exists(fp):
        return None
    with open(fp, newline="", encoding="utf-8") as f:
        rows = [r for r in csv.DictReader(f) if r["Name"].startswith(kernel_prefix)]
    if not rows:
        return None
    calls = sum(int(r["Calls"]) for r in rows)
    return sum(float(r["TotalDurationNs"]) for r in rows) / calls / 1e6


def _window_trace(kernel: str, args):
    """The committed kernel-trace window averages (profiles/r06_window_trace.json, tools/window_avg.py)
    when they were taken with this run's warmup / steps / sims / games, else None."""
    fp = os.path.join(ROOT, "profiles", "r06_window_trace.json")
    try:
        with open(fp, encoding="utf-8") as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if (d.get("warmup"), d.get("steps"), d.get("sims"), d.get("games", args.games)) != (args.warmup, args.steps,
                                                                                          args.sims, args.games):
        return None
    k = d.get("kernels", {}).get(kernel)
    if not k or not k.get("window_avg_us"):
        return None
    return dict(k, source=os.path.basename(fp))


def _pmc_traffic(kernel_prefix: str, units_per_launch: int, with_source: bool = False):
    """HBM bytes per launch from the committed rocprofv3 PMC summaries (profiles/*pmc*.json) of this
    kernel at this launch size, FETCH_SIZE doubled per the gfx950 correction (MI355X_MICROARCH.md
    §HBM). Among the files holding the kernel at that size, the one with the highest "round" field
    wins (file names break ties only within a round). None when absent. with_source: (bytes, the
    profile's file name) — a committed measurement, not one of this run."""
    best = None
    for fp in glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")):
        try:
            with open(fp, encoding="utf-8") as f:
                d = json.load(f)
            k = d.get("kernels", {}).get(kernel_prefix)
            if k and k.get("units_per_launch") == units_per_launch:
                rank = (int(d.get("round", 0)), os.path.basename(fp))
                if best is None or rank > best[0]:
                    best = (rank, float(k["hbm_bytes_per_launch"]), os.path.basename(fp))
        except Exception:
            continue
    if best is None:
        return (None, None) if with_source else None
    return (best[1], best[2]) if with_source else best[1]


# ----------------------------------------------------------------------------- CPU baselines
# The reference-equivalent CPU paths (oracle/: the C restatement of the rules and the Python
# restatement of mcts.py) on every host core the box gives this job: one worker process per core
# ("one game per process on all host cores"), started before the benchmark touches
# the GPU (spawned, idle until the GPU legs are done), each running its own bounded sample.

def cpu_workers() -> int:
    """Host cores for the CPU baselines: BK_CPU_WORKERS, else the cores this process may run on,
    capped at 12: a GPU box gives one GPU 16 cores and lets at most 16 processes hold the GPU
    (a worker that imports torch counts, and the resnet baseline's workers do use it), so 12
    workers + this process stay inside both (nproc there shows the whole machine)."""
    n = os.environ.get("BK_CPU_WORKERS")
    if n:
        return max(1, int(n))
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    return max(1, min(12, avail))


def start_cpu_pool(n: int):
    import multiprocessing as mp

    return mp.get_context("spawn").Pool(n)


def stop_cpu_pool(args) -> None:
    """Join the CPU-baseline workers and end multiprocessing's resource tracker: the spawn pool's
    semaphores register with that helper process, which otherwise outlives the bench (the driver
    counted it as a leftover process, procs_at_end: 1). The pool must be unreferenced and collected
    first so its semaphores unregister before the tracker stops."""
    pool = getattr(args, "cpu_pool", None)
    if pool is None:
        return
    pool.close()
    pool.join()
    args.cpu_pool = None
    del pool
    import gc
    from multiprocessing import resource_tracker

    gc.collect()
    resource_tracker._resource_tracker._stop()


def _pool_run(pool, fn, jobs):
    """Run jobs (one per worker) concurrently -> (sum of units, max seconds, per-worker units)."""
    res = pool.map(fn, jobs) if pool is not None else [fn(j) for j in jobs]
    return sum(r[0] for r in res), max(r[1] for r in res), [r[0] for r in res]


def _w_legal(job):
    """Worker: legal masks of its share of the benchmark boards (C oracle), repeated for `seconds`."""
    states, seconds = job
    from oracle.oracle import Oracle

    o = Oracle(20, 4, 5)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o.legal_mask_batch(states)
        n += states.shape[0]
    return n, time.perf_counter() - t0


def _w_vecenv(job):
    seconds, seed = job
    from oracle.vecenv_oracle import VecEnvOracle

    ref = VecEnvOracle(64, 7, 4)
    ref.reset(seed)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for e in range(64):
            ref.step(e, -1)
        n += 64
    return n, time.perf_counter() - t0


def _w_config1(job):
    """Worker: 7x7 games from default_rng(seed) (uniform legal moves) to terminal on the C oracle,
    counting get_valid_moves + step calls."""
    cells, seed0, seconds = job
    from oracle.oracle import Oracle

    o = Oracle(7, 2, cells)
    calls, seed, t0 = 0, seed0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        rng = np.random.default_rng(seed)
        st = o.init_state()
        while o.game_ended(st) is None:
            ids = o.legal_ids(st)
            st, _ = o.next_state(st, int(ids[int(rng.integers(len(ids)))]))
            calls += 2
        seed += 1
    return calls, time.perf_counter() - t0


def _w_selfplay(job):
    """Worker: the reference-equivalent self-play of cpu_baseline_selfplay for `seconds`, its own
    game (moves sampled from pi at T=1 with default_rng(seed))."""
    seconds, model_type, seed = job
    return _selfplay_sample(seconds, model_type, seed)


def _selfplay_sample(seconds: float, model_type: str, seed: int):
    from blokus_rl_amd.nets import build_model
    from oracle.oracle import MCTSOracle, Oracle

    o = Oracle(20, 4, 5)
    torch.manual_seed(0)
    model = None
    if model_type != "dumbnet":
        torch.cuda.set_device(0)
        model = build_model(model_type, 20, 4, o.A, num_res_blocks=5).cuda().eval()

    def evaluate(s, player):
        ids = o.legal_ids(s, player)
        if model is None:
            return ids, np.full(len(ids), 1.0 / len(ids), dtype=np.float32), np.zeros(4)
        obs = torch.from_numpy(o.observe(s)).float().cuda().unsqueeze(0)
        mask = torch.zeros(o.A, dtype=torch.bool, device="cuda")
        mask[torch.from_numpy(ids).cuda()] = True
        with torch.inference_mode():
            lp, v = model(obs)
            p = torch.exp(torch.log_softmax(torch.masked_select(lp[0], mask), dim=-1))
        return ids, p.cpu().numpy(), v[0].cpu().numpy().astype(np.float64)

    rng = np.random.default_rng(seed)
    m = MCTSOracle(o, evaluate)
    s = o.init_state()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(100):
            m.simulate(s)
            n += 1
        ids, pi = m.get_distribution(s, 1)
        pi = np.asarray(pi, dtype=np.float64)
        s, _ = o.next_state(s, int(ids[int(rng.choice(len(ids), p=pi / pi.sum()))]))
        if o.game_ended(s) is not None:
            m = MCTSOracle(o, evaluate)
            s = o.init_state()
    return n, time.perf_counter() - t0


# ----------------------------------------------------------------------------- legal
def bench_legal(args, world, rank):
    from blokus_rl_amd.boards import random_boards
    from blokus_rl_amd.engine import Engine

    B = args.boards
    eng = Engine(20, 4, 5)
    states = random_boards(eng, B, seed0=rank * B)
    masks = torch.empty((B, eng.W), dtype=torch.int64, device=eng.device)
    counts = torch.empty(B, dtype=torch.int32, device=eng.device)
    stream = torch.cuda.current_stream()

    def step():
        eng.legal_mask_into(states, masks, counts)

    graph = None
    if args.graph:
        # capture `graph_steps` back-to-back passes; replay = graph_steps steps
        s = torch.cuda.Stream()
        s.wait_stream(stream)
        with torch.cuda.stream(s):
            step()
        stream.wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(args.graph_steps):
                step()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    _barrier(world)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    if graph is not None:
        reps = max(1, args.steps // args.graph_steps)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            graph.replay()
        e1.record(stream)
        steps_done = reps * args.graph_steps
    else:
        for i in range(args.steps):
            ev[i][0].record(stream)
            step()
            ev[i][1].record(stream)
        steps_done = args.steps
    torch.cuda.synchronize()
    _barrier(world)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    elapsed = _max_over_ranks(t1 - t0, world)
    if graph is not None:
        kernel_ms = e0.elapsed_time(e1) / steps_done
    else:
        kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    boards_total = B * steps_done * world
    value = boards_total / elapsed
    achieved = LEGAL_BYTES_PER_BOARD * B / (kernel_ms * 1e-3)
    traffic, traffic_src = _pmc_traffic("k_legal_mask", B, with_source=True)
    out = {
        "metric": "legal-move boards/sec (20x20, 4 players, 30433-id bitmask)",
        "value": value,
        "unit": "boards/s",
        "n_gpus": world,
        "steps": steps_done,
        "warmup": args.warmup,
        "ms_per_step": elapsed / steps_done * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32/u64 bitboards",
        "data": "synthetic: default_rng(b) random self-play boards, t~U{0..60} plies",
        "config": {"workload": "config 2: 20x20 legal-move enumeration, batch 4096 boards per GPU",
                   "global_batch": B * world, "parallelism": f"dp{world} (independent shards)",
                   "graph": bool(args.graph)},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK, "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "k_legal_mask", "kernel_ms": kernel_ms,
                     "bytes_per_unit": LEGAL_BYTES_PER_BOARD, "units_per_launch": B},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_legal(states, args.cpu_seconds, args.cpu_pool, args.cpu_workers)
    out["_states"] = states
    return out


def cpu_baseline_legal(states: torch.Tensor, seconds: float, pool=None, workers: int = 1):
    """The oracle (C restatement of the reference rules) on a bounded sample of the same boards:
    each worker repeats its share of the first 64 x workers boards until `seconds` pass."""
    sample = states[: 64 * workers].cpu().numpy()
    shares = [np.ascontiguousarray(x) for x in np.array_split(sample, workers)]
    n, dt, _ = _pool_run(pool, _w_legal, [(sh, seconds) for sh in shares])
    return {"value": n / dt, "unit": "boards/s", "cores": workers, "kind": "port",
            "sample": f"{n} board evaluations ({sample.shape[0]} benchmark boards split over {workers} worker "
                      f"processes, repeated) in {dt:.1f} s"}


# Config 5 bytes per env-step as k_vec_step7 moves them: the state words a 2-colour 7x7 game uses,
# read and written (occupancy rows 0..7 of colours 0 and 1, pieces, hash / to-move / ply, flags:
# 100 B each way), rng (16), obs (49 u8), mask (15 u64 = 120 at 919 ids), reward + done (8); the
# benchmark's agent draws in-kernel (no action read). DESIGN.md §4.
VEC_BYTES_PER_STEP = 100 + 100 + 16 + 49 + 120 + 8


def bench_vecenv(args, world, rank):
    """Config 5: the PPO 7x7 vector env, E envs, one fused k_vec_step7 launch per vector step;
    `value` from steps replayed out of a captured HIP graph (the device rate), plus the same steps
    called eagerly through env.step() and with masked policy sampling."""
    from blokus_rl_amd.vector_env import BlokusVectorEnv

    E = args.envs
    env = BlokusVectorEnv(E, 7, 4)
    env.reset(seed=rank)
    stream = torch.cuda.current_stream()
    for _ in range(20):
        env.step_raw(None)
    torch.cuda.synchronize()
    # the device step rate: the steps replayed from a HIP graph of `per` captured launches (the
    # host's per-call launch cost would otherwise set the rate of a ~10 us kernel)
    per = 25
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per):
            env.step_raw(None)
    g.replay()
    torch.cuda.synchronize()
    reps = max(1, args.vec_steps // per)
    _barrier(world)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(reps):
        g.replay()  # in-kernel random agent (policy stand-in), then the random opponent
    e1.record(stream)
    torch.cuda.synchronize()
    _barrier(world)
    dt = _max_over_ranks(time.perf_counter() - t0, world)
    steps_done = reps * per
    kernel_ms = e0.elapsed_time(e1) / steps_done
    # the same steps launched eagerly from Python, one env.step() call each (gymnasium-style API)
    torch.cuda.synchronize()
    te = time.perf_counter()
    for _ in range(200):
        env.step(None)
    torch.cuda.synchronize()
    eager = E * 200 / (time.perf_counter() - te)
    # PPO-style: the agent's actions drawn from policy logits each step (the rollout's
    # get_action_and_value + env.step, ppo/trainer.py:144-155) — the draw (FilterLegalMoves +
    # Categorical sample + log_prob) fused into k_vec_step7 (bk_vec_step_policy), replayed from a
    # HIP graph of `per` steps; the logits row is the actor's output stand-in (random, [E, A] f32 in
    # HBM). Beside it the draw alone (k_vec_policy, the standalone kernel).
    logits = (torch.randn((E, env.eng.A), device=env.device, generator=torch.Generator(env.device).manual_seed(rank))
              * 2.0).contiguous()
    gp, gs = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(gp):
        for _ in range(per):
            env.step_policy(logits)
    with torch.cuda.graph(gs):  # the draw alone (its kernel time for the roofline)
        for _ in range(per):
            env.sample_policy(logits)
    gp.replay()
    gs.replay()
    torch.cuda.synchronize()
    kbar = float(env.valid_mask().sum()) / E  # the agent's mean legal-id count on these boards
    reps2 = max(1, args.vec_steps // per)
    _barrier(world)
    t1 = time.perf_counter()
    e0.record(stream)
    for _ in range(reps2):
        gp.replay()
    e1.record(stream)
    torch.cuda.synchronize()
    _barrier(world)
    dt2 = _max_over_ranks(time.perf_counter() - t1, world)
    pair_ms = e0.elapsed_time(e1) / (reps2 * per)
    e0.record(stream)
    for _ in range(reps2):
        gs.replay()
    e1.record(stream)
    torch.cuda.synchronize()
    pol_ms = e0.elapsed_time(e1) / (reps2 * per)
    n2 = reps2 * per
    # the same draw as generic torch ops (the round-5 path): unpack the mask, -1e9 fill,
    # Categorical sample + log_prob, then env.step — for comparison only
    def torch_step():
        dist_t = torch.distributions.Categorical(logits=env.masked_logits(logits))
        a_t = dist_t.sample()
        dist_t.log_prob(a_t)
        env.step(a_t)

    for _ in range(3):
        torch_step()
    torch.cuda.synchronize()
    tt = time.perf_counter()
    for _ in range(50):
        torch_step()
    torch.cuda.synchronize()
    torch_ops = E * 50 / (time.perf_counter() - tt)
    # algorithmic bytes: the fused step = the env step's 393 B + the legal ids' logits (4 B each, the
    # only ones read) + the id and log-prob out; the standalone draw = its logits row reads of the
    # legal ids + the 120-B mask + rng 16 + out 8
    fused_bytes = VEC_BYTES_PER_STEP + 4.0 * kbar + 8
    pol_bytes = 4.0 * kbar + 8 * env.eng.W + 16 + 8
    achieved = VEC_BYTES_PER_STEP * E / (kernel_ms * 1e-3)
    # the headline is the DEVICE rate (graph-replayed launches, in-kernel agent draws); a gym-style
    # loop calling env.step() per step gets eager_env_step_calls (one launch + tensor bookkeeping
    # per call), and a PPO loop sampling from masked logits with_masked_policy_sampling
    out = {"metric": "PPO vector-env device steps/sec (7x7, 2 players, 919 ids, random opponent; HIP-graph-replayed "
                     "k_vec_step7 launches, in-kernel agent draws)",
           "value": E * steps_done * world / dt, "unit": "env-steps/s", "envs_per_gpu": E,
           "steps": steps_done, "eager_env_step_calls": {"value": eager * world, "unit": "env-steps/s"},
           "byte_accounting": "bytes_per_unit counts the state words a 7x7 game uses (393 B since round 4; "
                              "round 3 counted the whole 384-B state each way, 965 B): fractions are not "
                              "comparable with rounds <= 3",
           "with_masked_policy_sampling": {
               "value": E * n2 * world / dt2, "unit": "env-steps/s", "steps": n2,
               "path": "k_vec_step7<policy> (bk_vec_step_policy: FilterLegalMoves + Categorical sample + log_prob "
                       "fused into the env step), HIP-graph-replayed; logits [E, A] f32 resident in HBM (the actor's "
                       "output stand-in)",
               "ms_per_step": pair_ms, "legal_ids_per_env": kbar,
               "roofline": {"bound": "hbm", "kernel": "k_vec_step7<policy>",
                            "achieved": fused_bytes * E / (pair_ms * 1e-3) / 1e9, "peak": HBM_PEAK / 1e9,
                            "unit": "GB/s", "frac": fused_bytes * E / (pair_ms * 1e-3) / HBM_PEAK,
                            "kernel_ms": pair_ms, "bytes_per_unit": fused_bytes, "units_per_launch": E,
                            "traffic": _pmc_traffic("k_vec_step7_policy", E)},
               "draw_alone": {"kernel": "k_vec_policy", "kernel_ms": pol_ms, "bytes_per_unit": pol_bytes,
                              "achieved": pol_bytes * E / (pol_ms * 1e-3) / 1e9, "unit": "GB/s",
                              "frac": pol_bytes * E / (pol_ms * 1e-3) / HBM_PEAK,
                              "traffic": _pmc_traffic("k_vec_policy", E)},
               "torch_ops_eager": {"value": torch_ops, "unit": "env-steps/s",
                                   "note": "round-5 path: valid_mask + torch.where(-1e9) + Categorical.sample/log_prob + "
                                           "env.step per step"}},
           "roofline": {"bound": "hbm", "kernel": "k_vec_step7", "achieved": achieved / 1e9,
                        "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": achieved / HBM_PEAK,
                        "kernel_ms": kernel_ms, "bytes_per_unit": VEC_BYTES_PER_STEP, "units_per_launch": E,
                        "traffic": _pmc_traffic("k_vec_step7", E)}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_vecenv(args.cpu_seconds / 2, args.cpu_pool, args.cpu_workers)
    return out


def cpu_baseline_vecenv(seconds: float, pool=None, workers: int = 1):
    """The config-5 env restated on the CPU (oracle/vecenv_oracle.py: C oracle rules, Python
    loop per env like SyncVectorEnv), random agent + random opponent, 64 envs per worker."""
    n, dt, _ = _pool_run(pool, _w_vecenv, [(seconds, w) for w in range(workers)])
    return {"value": n / dt, "unit": "env-steps/s", "cores": workers, "kind": "port",
            "sample": f"{n} env steps of 64 sequential 7x7 envs per worker x {workers} workers in {dt:.1f} s"}


def cpu_baseline_selfplay(seconds: float, model_type: str = "resnet", pool=None, workers: int = 1):
    """Reference-equivalent CPU path: the pure-Python restatement of
    MCTS.simulate (oracle/oracle.py, float64, dict-keyed tree) and the C oracle env, one game per
    worker process on `workers` host cores; for resnet, batch-1 leaf evaluation of the unfused
    ResNet on the GPU with a host round trip per leaf exactly like BlokusNNetWrapper.predict
    (neural_network.py:92-110). 100 simulations per move, moves sampled from pi (T=1)."""
    n, dt, per = _pool_run(pool, _w_selfplay, [(seconds, model_type, w) for w in range(workers)])
    return {"value": n / dt, "unit": "sims/s", "cores": workers, "kind": "port",
            "per_core": float(np.mean(per)) / dt,
            "sample": f"{n} simulations ({model_type} leaf eval{' on the GPU, batch 1' if model_type != 'dumbnet' else ''}"
                      f"), one game per worker process x {workers} from the empty board, in {dt:.1f} s"}


def bench_config1(args, pool=None, workers: int = 1):
    """Config 1: 7x7 2-player games, get_valid_moves + step to terminal, uniform random legal moves
    from numpy default_rng(seed), for both 7x7 piece sets (2522 ids = all 21 pieces,
    as the recordings show; 919 ids = pieces of <= 4 cells, the documented gym action space).
    Engine legs: the drop-in ColosseumBlokusGameWrapper at batch 1 (each call a device round trip,
    the reference's calling pattern) and the batched engine (1024 games in lock-step on the GPU,
    device-side sampling). CPU leg: the C oracle, one worker process per host core."""
    from types import SimpleNamespace

    from blokus_rl_amd.colossumrl import ColosseumBlokusGameWrapper

    out = {"metric": "7x7 get_valid_moves + step calls/s (2 players, random legal moves to terminal)",
           "unit": "calls/s"}
    secs = max(1.0, args.cpu_seconds / 4)
    for cells in (5, 4):
        game = ColosseumBlokusGameWrapper(SimpleNamespace(board_size=7, number_of_players=2, max_piece_cells=cells))
        calls, games, seed, t0 = 0, 0, 0, time.perf_counter()
        while time.perf_counter() - t0 < secs:
            rng = np.random.default_rng(seed)
            s, p = game.get_init_board()
            while game.get_game_ended(s) is None:
                ids = np.nonzero(game.get_valid_moves(s, p))[0]
                s, p = game.get_next_state(s, p, int(ids[int(rng.integers(len(ids)))]))
                calls += 2
            games += 1
            seed += 1
        dt_drop = time.perf_counter() - t0
        eng = game.engine
        G = 1024
        gen = torch.Generator(device=eng.device).manual_seed(0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = eng.init_states(G)
        plies = torch.zeros((), dtype=torch.int64, device=eng.device)
        for i in range(4 * eng.num_pieces * eng.P):
            ids, cnt = eng.legal_ids(st, cap=1024)
            live = cnt > 0
            pick = (torch.rand(G, device=eng.device, generator=gen) * cnt.clamp(min=1)).long()
            act = torch.where(live, ids.gather(1, pick.view(-1, 1)).view(-1), torch.full_like(cnt, -1))
            st, _, _ = eng.next_state(st, act.to(torch.int32).contiguous())
            plies += live.sum()
            if i % 8 == 7 and not bool(live.any()):
                break
        torch.cuda.synchronize()
        dt_b = time.perf_counter() - t0
        nb = 2 * int(plies)
        rec = {"ids": eng.A,
               "engine_dropin_batch1": {"value": calls / dt_drop, "unit": "calls/s", "games": games},
               "engine_batched": {"value": nb / dt_b, "unit": "calls/s", "games": G,
                                  "note": "legal-id enumeration + next state of 1024 games per launch pair"}}
        if not args.no_cpu_baseline:
            n, dt, _ = _pool_run(pool, _w_config1, [(cells, 100000 * w, secs) for w in range(workers)])
            rec["cpu_baseline"] = {"value": n / dt, "unit": "calls/s", "cores": workers, "kind": "port",
                                   "sample": f"{n} calls of 7x7 random games (C oracle, default_rng seeds), "
                                             f"{workers} worker processes, {dt:.1f} s"}
        out[f"ids_{eng.A}"] = rec
    out["value"] = out["ids_2522"]["engine_batched"]["value"]
    return out


def bench_train(args, world, rank):
    """§8f row 1: the learner on the device path (samples/s over all ranks; DDP over RCCL)."""
    from blokus_rl_amd.alphazero.learner_bench import bench_learner
    from blokus_rl_amd.engine import Engine

    eng = Engine(20, 4, 5)
    res = {}
    # the learner's default ("auto": the device path at large batches), the same batch on the
    # fp32 MIOpen path, and the reference's batch 64
    for key, bs, dpath in (("main", args.train_batch, "auto"), ("fp32", args.train_batch, False), ("b64", 64, "auto")):
        r = bench_learner(eng, world, rank, bs, args.train_steps, 3, rows=args.train_rows,
                          reference_steps=0 if (args.no_cpu_baseline or key != "b64") else 10,
                          barrier=(lambda: _barrier(world)), device_path=dpath)
        dt = _max_over_ranks(r["elapsed_s"], world)
        r["value"] = bs * args.train_steps * world / dt
        r["unit"] = "samples/s"
        r["ms_per_step"] = dt / args.train_steps * 1e3
        res[key] = r
    main_r = res["main"]
    lk = main_r["loss_kernels"]
    out = {"metric": "AlphaZero learner samples/sec (20x20 ResNet-5x64, Adam, device replay batches)",
           "value": main_r["value"], "unit": "samples/s", "n_gpus": world, "steps": args.train_steps,
           "ms_per_step": main_r["ms_per_step"], "higher_is_better": True, "scaling": "weak",
           "dtype": "fp32 (tower convs: split-f16 x3 products, fp32-class)" if main_r["device_path"] else "fp32", "data": "synthetic replay: random-play boards, Dirichlet pi, one-hot z",
           "config": {"workload": "§8f row 1 learner", "batch_per_gpu": args.train_batch,
                      "global_batch": args.train_batch * world, "parallelism": f"ddp{world}"},
           "device_path": main_r["device_path"],
           "path": ("tower convs on trainconv.hip (forward + input gradient: k_conv_x3; weight gradient: "
                    "k_conv_x3_wgrad; split-f16 MFMA, fp32-class), the 64-channel train-mode batch norms on "
                    "trainbn.hip (k_bn_reduce / k_bn_axpb), channels_last; stem, heads and Adam on PyTorch"
                    if main_r["device_path"] else "fp32 MIOpen"),
           "fp32_miopen_same_batch": {k: res["fp32"][k] for k in ("value", "unit", "ms_per_step")},
           "at_reference_batch_64": {k: res["b64"][k] for k in ("value", "unit", "ms_per_step", "device_path")},
           "roofline": {"bound": "hbm", "kernel": lk["kernel"], "achieved": lk["achieved_GBps"],
                        "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": lk["achieved_GBps"] * 1e9 / HBM_PEAK,
                        "kernel_ms": lk["ms"], "bytes_per_launch_pair": lk["bytes_per_launch_pair"],
                        "units_per_launch": args.train_batch,
                        "traffic": _pmc_traffic("k_policy_loss+grad", args.train_batch)}}
    if "conv_kernel" in main_r:  # the device path's dominant kernel: k_conv_x3 on the f16 matrix cores
        ck = main_r["conv_kernel"]
        out["loss_roofline"] = out["roofline"]
        out["roofline"] = {"bound": "mfma", "kernel": ck["kernel"], "achieved": ck["flop"] / (ck["ms"] * 1e-3) / 1e12,
                           "peak": MFMA_F16_PEAK / 1e12, "unit": "TFLOP/s",
                           "frac": ck["flop"] / (ck["ms"] * 1e-3) / MFMA_F16_PEAK, "kernel_ms": ck["ms"],
                           "flop_per_launch": ck["flop"], "units_per_launch": args.train_batch,
                           "traffic": _pmc_traffic("k_conv_x3", args.train_batch),
                           "fp32_equiv_tflops": ck["fp32_equiv_flop"] / (ck["ms"] * 1e-3) / 1e12,
                           "frac_algorithmic": ck["fp32_equiv_flop"] / (ck["ms"] * 1e-3) / MFMA_F16_PEAK,
                           "note": "frac: executed split-f16 MFMA work (3 f16 products per fp32 product); "
                                   "frac_algorithmic: the fp32 conv's FLOP"}
        if "wgrad_kernel" in main_r:
            wk = main_r["wgrad_kernel"]
            out["wgrad_roofline"] = {"bound": "mfma", "kernel": wk["kernel"], "kernel_ms": wk["ms"],
                                     "achieved": wk["flop"] / (wk["ms"] * 1e-3) / 1e12, "peak": MFMA_F16_PEAK / 1e12,
                                     "unit": "TFLOP/s", "frac": wk["flop"] / (wk["ms"] * 1e-3) / MFMA_F16_PEAK,
                                     "frac_algorithmic": wk["fp32_equiv_flop"] / (wk["ms"] * 1e-3) / MFMA_F16_PEAK,
                                     "flop_per_launch": wk["flop"], "units_per_launch": args.train_batch,
                                     "traffic": _pmc_traffic("k_conv_x3_wgrad", args.train_batch)}
    if "reference_path" in res["b64"]:
        out["reference_path_batch_64"] = res["b64"]["reference_path"]
    return out


def bench_ppo(args, world, rank):
    """§8f row 4: whole PPO updates on the config-5 device env (reference config
    ppo_blokus_7x7.yml: cnn agent, d_model 128, 32 steps per rollout; 8192 envs per GPU): each
    update = the rollout (agent forward + bk_vec_policy + k_vec_step7 per step, ppo/trainer.py:128-175)
    + the GAE kernel (:177-211) + 4 epochs x 4 minibatches of the clipped update (:213-311).
    The agent's convolutions run on MIOpen (NCHW, fp32); the bench sets MIOPEN_FIND_MODE=FAST in its
    own process (`ppo_update_subprocess`): the default find mode spends ~160 s building kernels on a
    fresh box for the same steady-state update time (round 6: 157.5 s vs 4.5 s warm-up, 2.00 vs 2.03 s
    per update)."""
    from blokus_rl_amd.ppo.trainer import PPOHparams, PPOTrainer, compute_gae

    E, T = args.envs, 32
    hp = PPOHparams(num_envs=E, num_steps=T, agent_type="cnn", d_model=128, learning_rate=1e-5,
                    total_timesteps=E * T * 100, seed=rank, save_interval=10**9, target_kl=None)
    tr = PPOTrainer(hp)
    tw = time.perf_counter()
    tr.train(1)  # warm-up update (MIOpen's first-use kernel builds for the agent's convs land here)
    torch.cuda.synchronize()
    warm_s = time.perf_counter() - tw
    _barrier(world)
    t0 = time.perf_counter()
    n = args.ppo_updates
    tr.train(n)
    torch.cuda.synchronize()
    _barrier(world)
    dt = _max_over_ranks(time.perf_counter() - t0, world)
    # where an update's time goes (one more update with synchronizing phase timers; not in value)
    tr.phase_timers = True
    tr.train(1)
    phases = dict(tr.phase_s)
    dev = tr.device
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # the update's dominant kernel: the 128 -> 128 3x3 conv's input gradient at the minibatch size
    # (MIOpen igemm_bwd_gtcx35_nhwc fp32 on the f32 matrix cores, behind its NCHW -> NHWC transposes;
    # r06 kernel trace: profiles/r06_ppo_kernel_stats.csv), timed alone with events on the stream it
    # runs on (the event pair also holds the transposes)
    mb = hp.minibatch_size
    conv = tr.agent.conv_block.conv_block[3]
    xg = torch.randn((mb, hp.d_model, 7, 7), device=dev)
    xg.requires_grad_(True)
    yg = conv(xg)
    dyg = torch.randn_like(yg)
    for _ in range(2):
        torch.autograd.grad(yg, xg, dyg, retain_graph=True)
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(5):
        torch.autograd.grad(yg, xg, dyg, retain_graph=True)
    e1.record(st)
    torch.cuda.synchronize()
    dgrad_ms = e0.elapsed_time(e1) / 5
    conv_flop = 2.0 * mb * 49 * hp.d_model * hp.d_model * 9
    del xg, yg, dyg
    # the GAE kernel alone on this rollout
    m = tr.memory
    nv = torch.zeros(E, device=dev)
    compute_gae(m.rewards, m.values, m.dones, nv, nv, 0.99, 0.95)
    e0.record(st)
    for _ in range(20):
        compute_gae(m.rewards, m.values, m.dones, nv, nv, 0.99, 0.95)
    e1.record(st)
    torch.cuda.synchronize()
    gae_ms = e0.elapsed_time(e1) / 20
    gae_bytes = 5 * T * E * 4 + 2 * E * 4
    out = {"metric": "PPO env-steps/sec incl. updates (7x7 cnn agent d_model 128, 32-step rollouts, 4 x 4 minibatches)",
           "value": E * T * n * world / dt, "unit": "env-steps/s", "envs_per_gpu": E, "updates": n,
           "updates_per_s": n / dt, "s_per_update": dt / n, "warmup_update_s": warm_s,
           "miopen_find_mode": os.environ.get("MIOPEN_FIND_MODE"), "dtype": "fp32",
           "phase_s_one_update": phases,
           "last_log": {k: float(v) for k, v in tr.logs[-1].items()},
           "roofline": {"bound": "mfma", "kernel": "MIOpen igemm_bwd (conv 128->128 3x3 input gradient, fp32, with its NCHW<->NHWC transposes)",
                        "achieved": conv_flop / (dgrad_ms * 1e-3) / 1e12, "peak": MFMA_F32_PEAK / 1e12,
                        "unit": "TFLOP/s", "frac": conv_flop / (dgrad_ms * 1e-3) / MFMA_F32_PEAK, "kernel_ms": dgrad_ms,
                        "flop_per_launch": conv_flop, "units_per_launch": mb, "traffic": None,
                        "kernel_only_ms_trace": _trace_avg_ms("r06_ppo_kernel_stats.csv", "igemm_bwd_gtcx35_nhwc_fp32"),
                        "kernel_only_trace_source": "r06_ppo_kernel_stats.csv",
                        "note": "one of the update's three equal-cost conv kernels (fwd / dgrad / wgrad, ~17% of the "
                                "update's GPU time each in the kernel trace); f32-input MFMA peak 157.3 TF"},
           "gae_kernel": {"ms": gae_ms, "bytes": gae_bytes, "achieved_GBps": gae_bytes / (gae_ms * 1e-3) / 1e9}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_ppo(hp)
    return out


def cpu_baseline_ppo(hp_gpu):
    """The reference's PPO iteration on the host cores at a bounded size: 64 envs of the CPU
    restatement (oracle/vecenv_oracle.py, a Python loop per env like SyncVectorEnv), the same cnn
    agent on the CPU (torch, all granted threads), FilterLegalMoves + Categorical per step
    (ppo/agent.py:27-42, 148-156), GAE (oracle/ppo_oracle.py) and one optimize_agent pass (4 epochs
    x 4 minibatches of 512): one whole update, timed."""
    import dataclasses

    from blokus_rl_amd.ppo.agent import get_agent
    from blokus_rl_amd.ppo.trainer import optimize_agent
    from oracle.ppo_oracle import filter_legal, gae_f32
    from oracle.vecenv_oracle import VecEnvOracle

    threads = cpu_workers()
    old_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        E, T = 64, hp_gpu.num_steps
        hp = dataclasses.replace(hp_gpu, num_envs=E)
        torch.manual_seed(0)
        agent = get_agent("cnn")((7, 7), 919, hp)
        opt = torch.optim.Adam(agent.parameters(), lr=hp.learning_rate, eps=hp.eps)
        env = VecEnvOracle(E, 7, 4)
        env.reset(0)
        obs = torch.zeros((T, E, 7, 7))
        acts, lps, vals, rews, dones = (torch.zeros((T, E)) for _ in range(5))
        t0 = time.perf_counter()
        nobs = torch.from_numpy(np.stack([env.obs(e) for e in range(E)])).float()
        ndone = torch.zeros(E)
        for t in range(T):
            obs[t], dones[t] = nobs, ndone
            with torch.inference_mode():
                h = agent.features(nobs)
                mask = np.zeros((E, 919), np.float32)
                for e in range(E):
                    m = env.mask(e)
                    mask[e] = np.unpackbits(m.view(np.uint8), bitorder="little")[:919]
                logits = torch.from_numpy(filter_legal(agent.actor(h).numpy(), mask))
                dist = torch.distributions.Categorical(logits=logits)
                a = dist.sample()
                lps[t], vals[t], acts[t] = dist.log_prob(a), agent.critic(h).view(-1), a.float()
            res = [env.step(e, int(a[e])) for e in range(E)]
            rews[t] = torch.tensor([r for r, _ in res])
            ndone = torch.tensor([float(d) for _, d in res])
            nobs = torch.from_numpy(np.stack([env.obs(e) for e in range(E)])).float()
        with torch.inference_mode():
            nv = agent.get_value(nobs).view(-1).numpy()
        adv, ret = gae_f32(rews.numpy(), vals.numpy(), dones.numpy(), nv, ndone.numpy(), hp.gamma, hp.gae_lambda)
        batch = {"obs": obs.reshape(-1, 7, 7), "logprobs": lps.reshape(-1), "actions": acts.reshape(-1),
                 "advantages": torch.from_numpy(adv).reshape(-1), "returns": torch.from_numpy(ret).reshape(-1),
                 "values": vals.reshape(-1)}
        t1 = time.perf_counter()
        optimize_agent(agent, opt, batch, hp)
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(old_threads)
    return {"value": E * T / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"one whole PPO update at 64 envs x {T} steps (rollout {t1 - t0:.1f} s: C-oracle envs in a Python "
                      f"loop + the cnn agent on {threads} CPU threads; update {dt - (t1 - t0):.1f} s: 4 epochs x 4 "
                      f"minibatches of 512) in {dt:.1f} s"}


def ppo_update_subprocess(args):
    """The PPO leg of the default run in a child process of its own (MIOPEN_FIND_MODE=FAST there
    only, so MIOpen's other users in this process keep the default mode); its JSON line back."""
    import subprocess

    cmd = [sys.executable, os.path.abspath(__file__), "--workload", "ppo", "--ppo-updates", str(args.ppo_updates),
           "--envs", str(args.envs)] + (["--no-cpu-baseline"] if args.no_cpu_baseline else [])
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                            "MASTER_PORT", "BK_DIST_BACKEND")}
    env["MIOPEN_FIND_MODE"] = "FAST"
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=args.ppo_timeout, check=False)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode == 0 and lines:
            return json.loads(lines[-1])
        return {"error": f"exit {r.returncode}", "stderr_tail": r.stderr[-800:]}
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {args.ppo_timeout} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["all", "legal", "selfplay", "vecenv", "train", "ppo", "dry"],
                    default="all")
    ap.add_argument("--ppo-updates", type=int, default=2)
    ap.add_argument("--ppo-timeout", type=float, default=240.0)
    ap.add_argument("--train-batch", type=int, default=1024)
    ap.add_argument("--train-steps", type=int, default=20)
    ap.add_argument("--train-rows", type=int, default=8192)
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--vec-steps", type=int, default=1000)
    ap.add_argument("--legal-steps", type=int, default=200)
    ap.add_argument("--legal-warmup", type=int, default=20)
    ap.add_argument("--boards", type=int, default=4096)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--graph-steps", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--late-plies", type=int, default=30,
                    help="self-play: plies timed after the window (the late game; 0 = skip), sub-field late_game")
    ap.add_argument("--games", type=int, default=256)
    ap.add_argument("--sims", type=int, default=100)
    ap.add_argument("--model", default="resnet", choices=["resnet", "dumbnet", "dcnnet"])
    ap.add_argument("--nn-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--node-cap", type=int, default=None,
                    help="nodes per tree (default: sims x the longest game + 1, SelfPlay.node_cap_for)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process started with --gpus N: become the launcher of N ranks (nothing here has
        # touched the GPU; the ranks are child processes, not an exec of this one)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    args.cpu_workers, args.cpu_pool = 1, None
    if (not args.no_cpu_baseline and int(os.environ.get("WORLD_SIZE", "1")) == 1 and args.workload != "dry"
            and args.workload not in ("train", "ppo")):
        # the CPU-baseline worker processes, started before anything touches the GPU
        args.cpu_workers = cpu_workers()
        args.cpu_pool = start_cpu_pool(args.cpu_workers) if args.cpu_workers > 1 else None
    world, rank, _ = _dist_init(need_gpu=args.workload != "dry")
    if args.workload == "dry":
        out = bench_dry(args, world, rank)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if dist_active():
            dist.destroy_process_group()
        return
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; reporting the {world} ranks that run",
              file=sys.stderr)
    if args.workload == "legal":
        out = bench_legal(args, world, rank)
    elif args.workload == "vecenv":
        out = bench_vecenv(args, world, rank)
    elif args.workload == "train":
        out = bench_train(args, world, rank)
    elif args.workload == "ppo":
        out = bench_ppo(args, world, rank)
    else:
        from blokus_rl_amd.alphazero.selfplay_bench import bench_selfplay, run_selfplay
        out = bench_selfplay(args, world, rank)
        sr = out.get("search_roofline", {})
        if "k_leaf_step" in sr.get("kernel", ""):
            # the leaf step's time over the timed window: the average over the window's launches in
            # the committed kernel trace of this same command (profiles/r06_window_trace.json,
            # tools/window_avg.py), beside this run's live sample after the window; HBM-side bytes
            # per launch from the committed PMC passes over the same window: the fraction of the
            # HBM roofline it draws (committed profiles, named as such)
            sr["k_leaf_step_us_live_after_window"] = sr.pop("k_leaf_step_us", None)
            win = _window_trace("k_leaf_step_ov", args)
            sr["k_leaf_step_us"] = win["window_avg_us"] if win else sr["k_leaf_step_us_live_after_window"]
            sr["k_leaf_step_us_source"] = (f"kernel-trace average over the window's {win['window_dispatches']} "
                                           f"launches, {win['source']}" if win else "live sample after the window")
            tr, src = _pmc_traffic("k_leaf_step_ov", args.games, with_source=True)
            sr["traffic"], sr["traffic_source"] = tr, src
            if tr and sr.get("k_leaf_step_us"):
                sr["achieved_est"] = tr / (sr["k_leaf_step_us"] * 1e-6) / 1e9
                sr["frac_est"] = sr["achieved_est"] / sr["peak"]
        tw = _window_trace("k_leafnet_x3", args)
        if tw and "tower_roofline" in out:
            out["tower_roofline"]["kernel_ms_window_trace"] = tw["window_avg_us"] / 1e3
            out["tower_roofline"]["kernel_ms_window_trace_source"] = tw["source"]
        kname = out["roofline"].get("kernel", "").split(" ")[0]
        if kname.startswith("k_conv3x3") or kname.startswith("k_tower") or kname.startswith("k_leafnet"):
            # HBM bytes per launch from the committed PMC passes (profiles/r01_pmc_conv*.json)
            out["roofline"]["traffic"], out["roofline"]["traffic_source"] = _pmc_traffic(kname, args.games, True)
        if args.workload == "all" and args.model == "resnet" and args.nn_dtype == "fp32":
            # the same self-play with the leaf net at the reference's own precision: every product
            # on the exact-f32 MFMA (BK_NET_MATH=f32), timed the same way
            from blokus_rl_amd.nets import net_math

            if net_math() == "x3":
                os.environ["BK_NET_MATH"] = "f32"
                try:
                    _, _, fsims, fdt, _, _ = run_selfplay("resnet", "fp32", args.games, args.sims, args.steps,
                                                          args.warmup, rank, args.node_cap, world, timers=False)
                finally:
                    del os.environ["BK_NET_MATH"]
                out["net_math_f32"] = {"value": _sum_over_ranks(fsims, world) / _max_over_ranks(fdt, world),
                                       "unit": "sims/s", "dtype": "fp32 net: exact f32 MFMA products "
                                       "(v_mfma_f32_16x16x4_f32, Winograd F(2x2,3x3) tower), BK_NET_MATH=f32"}
        if args.workload == "all":
            # env + search alone: the uninformed-MCTS opponent (DumbNet, compare_arena.py:87-95)
            _, _, dsims, dt, dctr, dms = run_selfplay("dumbnet", "fp32", args.games, args.sims, args.steps,
                                                      args.warmup, rank, args.node_cap, world)
            dsims_all = _sum_over_ranks(dsims, world)
            out["uninformed_mcts"] = {"value": dsims_all / _max_over_ranks(dt, world), "unit": "sims/s",
                                      "stage_ms_per_sim_step": dms, "engine_counters": dctr}
            largs = argparse.Namespace(**vars(args))
            largs.steps, largs.warmup, largs.no_cpu_baseline = args.legal_steps, args.legal_warmup, True
            legal = bench_legal(largs, world, rank)
            out["legal_move"] = {k: legal[k] for k in ("metric", "value", "unit", "ms_per_step", "steps", "roofline")}
            vargs = argparse.Namespace(**vars(args))
            vargs.no_cpu_baseline = True
            out["ppo_vector_env"] = bench_vecenv(vargs, world, rank)
            out["learner"] = bench_train(args, world, rank)
            if world == 1:
                out["config1_7x7"] = bench_config1(args, args.cpu_pool, args.cpu_workers)
                out["ppo_update"] = ppo_update_subprocess(args)
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            pool, nw = args.cpu_pool, args.cpu_workers
            out["cpu_baseline"] = cpu_baseline_selfplay(args.cpu_seconds, args.model, pool, nw)
            if args.workload == "all":
                out["cpu_baseline_uninformed"] = cpu_baseline_selfplay(args.cpu_seconds / 2, "dumbnet", pool, nw)
                out["legal_move"]["cpu_baseline"] = cpu_baseline_legal(legal["_states"], args.cpu_seconds / 2, pool, nw)
                out["ppo_vector_env"]["cpu_baseline"] = cpu_baseline_vecenv(args.cpu_seconds / 2, pool, nw)
    out.pop("_states", None)
    pool = largs = vargs = None  # (the Namespace copies hold the pool too)
    stop_cpu_pool(args)
    if dist_active():
        out["dist_backend"] = dist.get_backend()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_active():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
