"""bench.py --workload selfplay: AlphaZero self-play sims/s (BASELINE.json configs 3 and 4).

Per GPU: 256 concurrent 4-player 20x20 games, 100 MCTS simulations per move, cpuct 1,
temperature 1, first-ply Dirichlet(1) x 0.25, ResNet (5 blocks, 64 channels, A=30433,
24.78M params) with random-init weights (seed 0) as the leaf evaluator. A step = one ply of
every game (= 256 x 100 simulations). Ranks play independent games (seeded by rank).
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist


from ..engine import Engine
from ..nets import build_model
from ..replay import dist_active
from .selfplay import SelfPlay

FP32_PEAK = 157.3e12             # MI355X_MICROARCH.md (f32 vector = f32 MFMA)
FP16_PEAK = 2.5e15               # dense bf16/fp16 MFMA
HBM_PEAK = 8.0e12


def search_bytes(c: dict, sims: int, obs_bytes: int, mask_bytes: int) -> float:
    """Algorithmic HBM bytes of the search kernels (k_select + k_expand_backup) from engine
    counters: root state read per simulation; per descended level
    16 B x K child stats + 52 B (hash probe, node header, child id, path record) + 40 B backup;
    per expanded leaf the state, bitmask and observation row written, the bitmask re-read, 36 B
    of node/value; per created child 4 B logit gather + 20 B child init."""
    return (sims * 384 + c["scanned"] * 16 + c["levels"] * (52 + 40)
            + c["expanded"] * (384 + mask_bytes + obs_bytes + mask_bytes + 36) + c["leaf_children"] * 24)


def leaf_step_bytes(c: dict, sims: int, N: int, P: int, W64: int, F: int) -> float:
    """Algorithmic bytes of a sim-step's search launches on the timed path (k_select once per ply,
    then k_leaf_step per simulation) from engine counters, as the kernels move them:
    per simulation the root state (384); per descended level one 64-entry table probe (1 KB), the
    node's child statistics (20 B each: P, N, Q, id), the path record (12) and its backup (24);
    per expanded leaf the probe + entry (1040), the leaf state written and re-read (768), the legal
    bitmask written and re-read (2 x 8 W64), the observation (4 x 2P N^2), the policy features
    (4 F) and the value (16); per legal id of an expanded leaf its policy-Linear row and bias
    (4 F + 4: the sparse head, rows shared between trees are counted per use) and the child
    initialised (20)."""
    return (sims * 384 + c["levels"] * (1024 + 12 + 24) + c["scanned"] * 20
            + c["expanded"] * (1040 + 768 + 2 * 8 * W64 + 4 * 2 * P * N * N + 4 * F + 16)
            + c["leaf_children"] * (4 * F + 4 + 20))


def time_leaf_step(sp, n: int = 10):
    """The search half of the timed path, live: one eager k_select, then n x {leaf net (graph
    replay), k_leaf_step} with HIP events on the launch stream around each search launch (the
    same kernels the captured ply graph replays). -> dict(ms per sim-step of the search
    launches, bytes per sim-step, k_leaf_step us) or None (no sparse HIP net)."""
    ev = sp.evaluator
    if not ev.sparse or ev.graph is None:
        return None
    st = torch.cuda.current_stream(sp.eng.device)
    E = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    torch.cuda.synchronize()
    c0 = sp.mcts.counters()
    e_sel = (E(), E())
    e_sel[0].record(st)
    _, obs, _ = sp.mcts.select(sp.roots, sp.active, sp.cpuct)
    e_sel[1].record(st)
    steps = []
    for i in range(n):
        out, v = ev(obs)
        a, b = E(), E()
        a.record(st)
        last = i == n - 1
        sp.mcts.leaf_step(out, ev.policy_w, ev.policy_b, v, None if last else sp.roots, sp.active, sp.cpuct)
        b.record(st)
        steps.append((a, b))
    torch.cuda.synchronize()
    c1 = sp.mcts.counters()
    d = {k: c1[k] - c0[k] for k in c1 if k not in ("errors", "nodes", "children")}
    sel_ms = e_sel[0].elapsed_time(e_sel[1])
    step_ms = [a.elapsed_time(b) for a, b in steps]
    eng = sp.eng
    F = ev.policy_w.shape[1]
    active = int(sp.active.sum())
    nbytes = leaf_step_bytes(d, active * n, eng.N, eng.P, eng.W, F)
    return {"ms_per_sim_step": (sel_ms + sum(step_ms)) / n, "bytes_per_sim_step": nbytes / n,
            "k_leaf_step_us": 1e3 * sum(step_ms) / n, "k_select_us": 1e3 * sel_ms, "counters": d}


def run_selfplay(model_type: str, nn_dtype: str, G: int, sims: int, steps: int, warmup: int, rank: int,
                 node_cap: int, world: int, timers: bool = True):
    torch.manual_seed(0)
    eng = Engine(20, 4, 5)
    model = build_model(model_type, 20, 4, eng.A, num_res_blocks=5).to(eng.device).eval()
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[nn_dtype]
    sp = SelfPlay(eng, model, G, num_sims=sims, seed=1234 + rank, nn_dtype=dt, node_cap=node_cap, continuous=True)
    for _ in range(warmup):
        sp.play_ply()
    torch.cuda.synchronize()
    if dist_active():
        dist.barrier()
    torch.cuda.synchronize()
    c0 = sp.mcts.counters()
    sims0 = sp.stats.sims
    sp.mark_window()
    gather = {}
    t0 = time.perf_counter()
    for _ in range(steps):
        sp.play_ply()
    if dist_active():
        # config 4: the (s, pi, z) rows of the timed plies, all-gathered over RCCL/xGMI
        from ..replay import all_gather_packed

        tg = time.perf_counter()
        buf, cap = sp.window_packed()
        rows, _ = all_gather_packed(buf, cap)
        torch.cuda.synchronize()
        gather = {"rows_sent": int(buf.shape[0]), "rows_received": int(rows.shape[0]),
                  "bytes_received": int(rows.numel()), "seconds": time.perf_counter() - tg}
    torch.cuda.synchronize()
    if dist_active():
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    c1 = sp.check()  # raises on a node/child-table overflow or a root above cap
    done = sp.stats.sims - sims0
    delta = {k: c1[k] - c0[k] for k in c1 if k not in ("errors", "nodes", "children")}
    ms = stage_times(sp) if timers else {}
    if gather:
        ms["all_gather"] = gather
    return sp, eng, done, elapsed, delta, ms


def late_game(sp, plies: int, done: int) -> dict:
    """After the timed window (and the stage-timed ply): `plies` more plies of the same run,
    timed (sims/s and ms per ply of this rank; games that end restart, as in the window), then the
    live leaf-step time there — the window covers plies 5-30 of a ~60-80-ply game, this the rest
    (SURVEY §8d asks for the whole game's plies). {} when plies <= 0."""
    if plies <= 0:
        return {}
    torch.cuda.synchronize()
    sims0 = sp.stats.sims
    t0 = time.perf_counter()
    for _ in range(plies):
        sp.play_ply()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    sp.check()
    out = {"plies": f"{done + 1}-{done + plies}", "sims_per_s": (sp.stats.sims - sims0) / dt,
           "ms_per_ply": dt / plies * 1e3}
    ls = time_leaf_step(sp)
    if ls is not None:
        out["k_leaf_step_us"] = ls["k_leaf_step_us"]
    return out


def stage_times(sp) -> dict:
    """Stage times outside the timed region: one ply launched stage by stage with events around
    each stage: select / net / expand ms per sim-step."""
    out = {}
    sp.enable_timers(True)
    sp.play_ply()
    out.update(sp.timer_ms())
    sp.enable_timers(False)
    return out


def time_leaf_conv(sp, reps: int = 5):
    """The dominant kernel of the self-play step, timed live with HIP events on the stream it is
    launched on: `reps` eager forwards of the leaf net on the search's last leaf batch (the
    graph-captured forward is the same kernel sequence), one event pair around each launch of
    k_tower_wino (the fused residual tower + heads, bk_resnet_tower_heads) or, when the tower runs per layer
    (BK_TOWER=0 or an unsupported board size), around each residual-block k_conv3x3 launch.
    -> dict(ms per launch, FLOP per launch, kernel name, direct-conv FLOP per launch, launches per
    leaf batch) or None (no HIP ResNet). FLOP = the arithmetic the kernel's MFMAs execute: for the
    Winograd F(2x2,3x3) form 2*16*64*64 per 2x2 output tile and conv (16 transform-domain GEMMs),
    for the direct form 2*9*64*64 per output pixel and conv."""
    from .. import nets
    from ..engine import load_library
    from ..nets import LeafResNet

    model = getattr(sp.evaluator, "model", None)
    if not isinstance(model, LeafResNet) or not model.native or not len(model.f.blocks):
        return None
    G, N = sp.G, sp.eng.N
    nconv = 2 * len(model.f.blocks)
    obs = sp.evaluator.static_obs
    st = torch.cuda.current_stream(sp.eng.device)
    events = []
    orig_conv, orig_tower, orig_th = nets.conv3x3, nets.resnet_tower, nets.resnet_tower_heads
    orig_sth, orig_x3 = nets.resnet_stem_tower_heads, nets.leafnet_x3

    def timed(fn):
        def run(*a, **k):
            if fn is orig_conv and a[0].shape[1] != 64:  # the stem (planar observation input)
                return fn(*a, **k)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            y = fn(*a, **k)
            e1.record(st)
            events.append((e0, e1, fn is not orig_conv, fn is orig_sth or fn is orig_x3, fn is orig_x3))
            return y
        return run

    nets.conv3x3, nets.resnet_tower, nets.resnet_tower_heads = timed(orig_conv), timed(orig_tower), timed(orig_th)
    nets.resnet_stem_tower_heads, nets.leafnet_x3 = timed(orig_sth), timed(orig_x3)
    try:
        model(obs)  # warm
        events.clear()
        for _ in range(reps):
            model(obs)
    finally:
        nets.conv3x3, nets.resnet_tower, nets.resnet_tower_heads = orig_conv, orig_tower, orig_th
        nets.resnet_stem_tower_heads, nets.leafnet_x3 = orig_sth, orig_x3
    torch.cuda.synchronize()
    if not events:
        return None
    fused, with_stem, x3 = events[0][2], events[0][3], events[0][4]
    ms = sum(ev[0].elapsed_time(ev[1]) for ev in events) / len(events)
    layers = nconv if fused else 1
    stem = 2.0 * G * N * N * 64 * 9 * model.f.stem.in_channels if with_stem else 0.0
    direct = 2.0 * G * N * N * 64 * 9 * 64 * layers + stem
    if x3:
        # k_leafnet_x3: per board, layer and 16-pixel group, 3 f16 MFMAs 16x16x32 per K chunk of 32 in
        # each of the 4 waves (K = 9*64 = 576: 18 chunks; the stem's 72 padded to 96: 3 chunks)
        ng = (N * N + 15) // 16
        per_mfma = 2.0 * 16 * 16 * 32
        flop = G * 4 * ng * 3 * per_mfma * (18 * nconv + 3)
        return {"ms": ms, "flop": flop, "direct": direct, "launches": 1, "peak": FP16_PEAK,
                "kernel": "k_leafnet_x3 (the leaf ResNet in one launch, one workgroup per board: the stem and %d "
                          "direct 3x3 convs 64->64 as f16 MFMA 16x16x32 on split operands, 3 products per fp32 "
                          "product, f32 accumulation; bias/ReLU/residual, the heads' 1x1 convs and value MLP fused)"
                          % nconv}
    if load_library().bk_conv3x3_form(N, 64) == 1:
        flop = 2.0 * 16 * 64 * 64 * G * (N // 2) ** 2 * layers + stem
        name = ("k_tower_wino (the leaf ResNet in one launch, one workgroup per board: %sthe residual tower of "
                "%d Winograd F(2x2,3x3) f32 MFMA convs 64->64 with bias/ReLU/residual fused, the heads' 1x1 convs and "
                "value MLP)" % ("the stem conv (direct, f32 MFMA), " if with_stem else "", nconv) if fused else
                "k_conv3x3_wino2 (Winograd F(2x2,3x3), f32 MFMA, 64->64, fused bias+ReLU)")
    else:
        flop, name = direct, "k_conv3x3 (direct, f32 MFMA, 64->64, fused bias+ReLU)"
    return {"ms": ms, "flop": flop, "kernel": name, "direct": direct, "launches": 1 if fused else nconv,
            "peak": FP32_PEAK}


def net_dtype(args) -> str:
    from ..nets import net_math

    if args.nn_dtype == "fp32" and args.model == "resnet" and net_math() == "x3":
        return ("fp32 net (fp32 operands split into f16 hi+lo, 3 f16 MFMA products, f32 accumulation: fp32-class "
                "error, tests/test_leafnet_gpu.py) / f64 search / u32 bitboards")
    return f"{args.nn_dtype} net / f64 search / u32 bitboards"


def bench_selfplay(args, world, rank):
    G = args.games
    sp, eng, sims, elapsed, delta, ms = run_selfplay(args.model, args.nn_dtype, G, args.sims, args.steps,
                                                     args.warmup, rank, args.node_cap, world)
    local_sims = sims
    if dist_active():
        t = torch.tensor([elapsed, float(sims)], dtype=torch.float64, device="cuda")
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t)
        elapsed, sims = float(tmax[0].item()), int(t[1].item())
    steps_sim = args.steps * args.sims  # sim-steps timed (one simulation per tree each)
    obs_bytes = 4 * 2 * eng.P * eng.N * eng.N
    conv = time_leaf_conv(sp) if args.nn_dtype == "fp32" else None
    ls = time_leaf_step(sp)
    if ls is not None:
        # the search launches of the timed path (k_select + k_leaf_step), timed live
        # not an HBM-bound kernel: a chain of dependent L2/MALL round trips (the descent) beside a
        # gather that L2 mostly serves (PMC: about a third of the addressed bytes leave L2). So the
        # line carries the bytes as the kernels address them (policy-Linear rows counted per use)
        # as `addressed_*`, and the HBM fraction only from the measured HBM-side bytes per launch
        # (`traffic`, attached by bench.py from the committed PMC passes) over the live launch time
        addressed = ls["bytes_per_sim_step"] / (ls["ms_per_sim_step"] * 1e-3)
        search = {"bound": "latency/L2", "kernel": "k_leaf_step_ov (per simulation: sparse policy head, "
                                                   "expand/backup, next descent + leaf bitmask/observation; "
                                                   "k_select once per ply)",
                  "achieved": None, "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": None, "traffic": None,
                  "addressed_bytes_per_sim_step": ls["bytes_per_sim_step"], "addressed_GBps": addressed / 1e9,
                  "search_ms_per_sim_step": ls["ms_per_sim_step"], "k_leaf_step_us": ls["k_leaf_step_us"],
                  "note": "achieved_est/frac_est = the HBM-side bytes per k_leaf_step_ov launch of a committed "
                          "rocprofv3 PMC pass (FETCH_SIZE x2 + WRITE_SIZE, traffic_source) over this run's live "
                          "launch time: an estimate, not a measurement of this run; addressed_* count the bytes "
                          "as the kernels address them (each W row per use)"}
    else:
        sbytes = search_bytes(delta, local_sims, obs_bytes, 8 * eng.W)
        search_ms = ms.get("select", 0.0) + ms.get("expand", 0.0)
        achieved = sbytes / steps_sim / (search_ms * 1e-3) if search_ms else 0.0
        search = {"bound": "hbm", "kernel": "k_select+k_expand_backup (search, stage-timed eager ply)",
                  "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": achieved / HBM_PEAK,
                  "traffic": None, "bytes_per_sim_step": sbytes / steps_sim, "search_ms_per_sim_step": search_ms}
    late = late_game(sp, getattr(args, "late_plies", 0), args.warmup + args.steps + 1)
    out = {
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
        "dtype": net_dtype(args),
        "data": "synthetic: continuous self-play from the empty board, random-init ResNet weights (seed 0)",
        "config": {"workload": "config 3 (N=1) / 4 (N=8): AlphaZero self-play 20x20, 256 concurrent games per GPU, "
                               "100 sims/move, ResNet-5x64 leaf eval", "global_batch": G * world,
                   "parallelism": f"dp{world} (independent games)", "model": args.model},
        "search_roofline": search,
        "stage_ms_per_sim_step": ms,
        "engine_counters": delta,
    }
    if late:
        out["late_game"] = late
    if conv is not None:
        cms, cflop, dflop, cpeak = conv["ms"], conv["flop"], conv["direct"], conv["peak"]
        out["tower_roofline"] = {"bound": "mfma", "kernel": conv["kernel"],
                           "achieved": cflop / (cms * 1e-3) / 1e12, "peak": cpeak / 1e12, "unit": "TFLOP/s",
                           "frac": cflop / (cms * 1e-3) / cpeak, "traffic": None, "kernel_ms": cms,
                           "flop_per_launch": cflop, "units_per_launch": G,
                           # the leaf's algorithmic work = the direct conv + heads
                           # arithmetic of the fp32 network (298.6 MFLOP per 20x20 leaf), whatever the
                           # kernel executes (x3: 3 f16 products per fp32 product)
                           "algorithmic_flop_per_launch": dflop,
                           "frac_algorithmic": dflop / (cms * 1e-3) / cpeak,
                           "frac_note": "frac = executed MFMA work / peak (3 f16 products per fp32 product on x3); "
                                        "frac_algorithmic = the fp32 network's conv FLOP / peak",
                           "direct_conv_equiv_tflops": dflop / (cms * 1e-3) / 1e12,
                           "launches_per_sim_step": conv["launches"],
                           "share_of_sim_step": conv["launches"] * cms / (elapsed / steps_sim * 1e3)}
        out["roofline"] = out["tower_roofline"]
    else:
        out["roofline"] = out["search_roofline"]
    return out
