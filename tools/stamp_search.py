"""Diagnostic: per-phase cycle shares of k_select / k_expand_backup from the BK_STAMPS build
(BK_LIB=blokus_rl_amd/_lib/diag/libblokus_hip_diag.so). Runs self-play plies with the bench's
ResNet leaf net (or, with --dumbnet, the uninformed search), then stamps 30 simulations.
Usage: python tools/stamp_search.py [plies (4)] [--dumbnet]"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from blokus_rl_amd import engine
from blokus_rl_amd.engine import Engine
from blokus_rl_amd.nets import DumbNet, build_model
from blokus_rl_amd.alphazero.selfplay import SelfPlay

eng = Engine(20, 4, 5)
torch.manual_seed(0)
net = DumbNet(20, 4, eng.A) if "--dumbnet" in sys.argv else build_model("resnet", 20, 4, eng.A, num_res_blocks=5)
sp = SelfPlay(eng, net.to(eng.device).eval(), 256, num_sims=100, seed=1234, continuous=True)
plies = int(next((a for a in sys.argv[1:] if a.isdigit()), "4"))
for _ in range(plies):
    sp.play_ply()
lib = engine.load_library()
lib.bk_debug_stamps.argtypes = [ctypes.c_void_p]
acc = {0: [], 1: []}
for _ in range(30):
    sp.simulate()
    torch.cuda.synchronize()
    buf = np.zeros((2, 4096, 8), dtype=np.uint64)
    assert lib.bk_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    for k in (0, 1):
        acc[k].append(buf[k, :256].astype(np.int64))
for k, names in ((0, ["load", "descent", "build_mask", "mask+state store", "obs write"]),
                 (1, ["mask load", "compact", "table", "softmax+init", "backup"])):
    a = np.stack(acc[k])  # [iters, T, 8]
    d = np.diff(a[:, :, :6], axis=2)
    tot = a[:, :, 5] - a[:, :, 0]
    print(["k_select", "k_expand_backup"][k], "median total cycles", int(np.median(tot)),
          "(s_memtime ticks); per launch: mean of the max over trees", int(tot.max(axis=1).mean()),
          "p90", int(np.percentile(tot, 90)))
    for i, n in enumerate(names):
        print(f"   {n:18s} median {int(np.median(d[:, :, i])):8d}  mean {d[:, :, i].mean():10.0f}")
    for i, n in enumerate(names):  # the slowest tree of each launch: its phase split
        sl = np.argmax(tot, axis=1)
        print(f"   slowest tree {n:14s} mean {np.mean(d[np.arange(len(sl)), sl, i]):10.0f}")
    if k == 0:  # the descent's parts, summed over its levels
        for n, v in (("  probe", a[:, :, 6]), ("  select_child", a[:, :, 7]), ("  place_action", np.stack(acc[1])[:, :, 7]),
                     ("  advance_turn", np.stack(acc[1])[:, :, 6])):
            print(f"   {n:18s} median {int(np.median(v)):8d}  mean {v.mean():10.0f}")
