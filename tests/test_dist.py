"""The N>1 path on CPU: two gloo ranks exchange packed replay examples (ragged row counts and
different caps) with all_gather_packed; every rank must receive every row bit-exactly."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _examples(rank: int):
    g = torch.Generator().manual_seed(100 + rank)
    E = 5 + 3 * rank
    K = 70 + 100 * rank
    states = torch.randint(0, 256, (E, 384), dtype=torch.uint8, generator=g)
    k = torch.randint(1, K + 1, (E,), generator=g).to(torch.int32)
    ids = torch.randint(0, 30433, (E, K), generator=g).to(torch.int16)
    pi = torch.rand((E, K), generator=g)
    col = torch.arange(K).unsqueeze(0)
    ids = torch.where(col < k.unsqueeze(1), ids, torch.full_like(ids, -1))
    pi = torch.where(col < k.unsqueeze(1), pi, torch.zeros_like(pi))
    z = torch.tensor([[3.0, -1.0, -1.0, -1.0]]).repeat(E, 1)
    player = torch.arange(E, dtype=torch.int32) % 4
    return states, ids, pi, k, z, player


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from blokus_rl_amd.replay import all_gather_packed, pack, unpack
    buf, cap = pack(*_examples(rank)[:5], player=_examples(rank)[5])
    rows, cmax = all_gather_packed(buf, cap)
    u = unpack(rows, cmax)
    ok = True
    off = 0
    for r in range(world):
        states, ids, pi, k, z, player = _examples(r)
        E, K = ids.shape
        sl = slice(off, off + E)
        ok &= torch.equal(u["states"][sl], states) and torch.equal(u["k"][sl], k)
        ok &= torch.equal(u["player"][sl], player) and torch.equal(u["z"][sl], z)
        ok &= torch.equal(u["ids"][sl, :K], ids) and torch.equal(u["pi"][sl, :K], pi)
        ok &= bool((u["ids"][sl, K:] == -1).all())
        off += E
    ok &= off == rows.shape[0]
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


def test_all_gather_packed_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def test_bench_launches_ranks_itself():
    """`python bench.py --gpus 2` started as ONE process (as the driver starts it) launches two
    ranks itself (torch.distributed.run, 127.0.0.1) and rank 0 prints one JSON line. The dry
    workload rehearses it on CPU over gloo: both ranks' replay rows reach rank 0."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--workload", "dry"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["ranks_seen"] == [0, 1] and out["value"] == 3 + 4
    assert out["rows_intact"]


def test_bench_dry_world8_rows_intact():
    """The config-4 rank count: `bench.py --gpus 8 --workload dry` launches 8
    gloo ranks on CPU; every rank's ragged shard (3 + r rows, caps 64 and 128) must reach rank 0
    through all_gather_packed bit for bit, in rank order."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", "--workload", "dry"],
                       capture_output=True, text=True, timeout=400, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["ranks_seen"] == list(range(8))
    assert out["rows_intact"] and out["value"] == sum(3 + r for r in range(8)) and out["common_cap"] == 128


def test_bench_cpu_pool_leaves_no_process():
    """bench.py's CPU-baseline pool ends with no child process left (the driver counted
    multiprocessing's resource tracker as a leftover: procs_at_end 1 in BENCH_r04)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import argparse, psutil, bench\n"
            "a = argparse.Namespace(cpu_pool=bench.start_cpu_pool(2))\n"
            "assert a.cpu_pool.map(abs, [-1, 2]) == [1, 2]\n"
            "bench.stop_cpu_pool(a)\n"
            "print(len(psutil.Process().children(recursive=True)))\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == "0"
    assert "leaked" not in r.stderr and "Traceback" not in r.stderr, r.stderr[-2000:]
