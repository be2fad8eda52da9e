"""The config-4 path with several ranks on the one GPU of a test box: `bench.py --gpus 2` launches
two ranks itself; with BK_DIST_BACKEND=gloo both ranks share cuda:0 (RCCL refuses two ranks on
one device), so this rehearses everything of the 8-GPU run except RCCL itself — the launcher,
per-rank game seeds, the timed plies, the all-gather of the (s, pi, z) rows and the max-over-
ranks timing."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_selfplay_two_ranks_one_gpu():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["BK_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "selfplay", "--games", "16",
           "--sims", "4", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=100, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    # 2 ranks x 16 games x 4 sims x 3 plies
    assert out["engine_counters"]["expanded"] + out["engine_counters"]["terminal"] >= 16 * 4 * 3 - 16 * 3
    assert abs(out["value"] * out["ms_per_step"] * 1e-3 * out["steps"] - 2 * 16 * 4 * 3) < 1e-6 * 2 * 16 * 4 * 3 + 1
    ag = out["stage_ms_per_sim_step"]["all_gather"]
    assert ag["rows_sent"] == 16 * 3 and ag["rows_received"] == 2 * ag["rows_sent"]


def _run_json(cmd, env, timeout):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_rccl_world1_allgather_and_ddp():
    """The config-4 collectives on a real device: a world-size-1 RCCL group on cuda:0 (fresh child
    process) gathers packed (s, pi, z) rows through all_gather_into_tensor bit-exactly and takes a
    DDP learner step whose gradients equal the same step's without DDP bit for bit."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    out = _run_json([sys.executable, os.path.join(ROOT, "tests", "rccl_world1.py")], env, 110)
    assert out["backend"] == "nccl" and out["world"] == 1
    assert out["allgather_rows"] == 96 and out["allgather_equal"]
    assert out["ddp"] == "DistributedDataParallel"
    assert abs(out["loss_ddp"] - out["loss_plain"]) <= 1e-6 * max(1.0, abs(out["loss_plain"]))
    # deterministic backward (cudnn.deterministic in the child): bit-identical gradients, and the
    # Adam steps of the two copies agree to 1e-6
    assert out["grad_max_rel_diff"] == 0.0
    assert out["param_max_abs_diff"] <= 1e-6


def test_bench_selfplay_rccl_world1():
    """`BK_DIST_BACKEND=nccl bench.py --gpus 1`: the N>1 code path of the self-play bench (the
    all-gather of the timed plies' rows inside the timed region, max-over-ranks timing) on RCCL."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["BK_DIST_BACKEND"] = "nccl"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--workload", "selfplay", "--games", "16",
           "--sims", "4", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    out = _run_json(cmd, env, 110)
    assert out["n_gpus"] == 1 and out["dist_backend"] == "nccl"
    ag = out["stage_ms_per_sim_step"]["all_gather"]
    assert ag["rows_sent"] == 16 * 3 and ag["rows_received"] == ag["rows_sent"]
