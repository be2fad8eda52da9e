"""Diagnostic: phase cycles of the fused k_leaf_step (BK_STAMPS build,
BK_LIB=blokus_rl_amd/_lib/diag/libblokus_hip_diag.so): logits, expand/backup, descent, leaf
bitmask + observation, per tree, over the simulations of a few self-play plies (bench config)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from blokus_rl_amd import engine
from blokus_rl_amd.engine import Engine
from blokus_rl_amd.nets import build_model
from blokus_rl_amd.alphazero.selfplay import SelfPlay

eng = Engine(20, 4, 5)
torch.manual_seed(0)
net = build_model("resnet", 20, 4, eng.A, num_res_blocks=5)
sp = SelfPlay(eng, net.to(eng.device).eval(), 256, num_sims=100, seed=1234, continuous=True)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    sp.play_ply()
torch.cuda.synchronize()
lib = engine.load_library()
lib.bk_debug_step_stamps.argtypes = [ctypes.c_void_p]
buf = np.zeros((4096, 16), dtype=np.uint64)
assert lib.bk_debug_step_stamps(buf.ctypes.data_as(ctypes.c_void_p)) == 0
a = buf[:256, :5].astype(np.int64)  # the last k_leaf_step launch
d = np.diff(a, axis=1)
tot = a[:, 4] - a[:, 0]
start = a[:, 0] - a[:, 0].min()
print("k_leaf_step (last launch) total cycles: median", int(np.median(tot)), "max", int(tot.max()),
      "| WG start spread (max - min)", int(start.max()), "| end of the last WG - first start", int((a[:, 4] - a[:, 0].min()).max()))
for i, n in enumerate(["logits+handoff", "expand+handoff", "descent", "bitmask+obs"]):
    print(f"  {n:16s} median {int(np.median(d[:, i])):8d}  max {int(d[:, i].max()):8d}")
m = buf[:256, :8].astype(np.int64)
for n, (i, j) in (("descent end -> ctx done (zero, row_ctx)", (3, 5)), ("first barrier", (5, 6)),
                  ("orientations (thread 0's wave)", (6, 7)), ("second barrier .. obs end", (7, 4))):
    print(f"  mask: {n:40s} median {int(np.median(m[:, j] - m[:, i])):8d}")
if "--twice" in sys.argv:
    print(f"  mask: orientations again (warm)  median {int(np.median(m[:, 3] - m[:, 7])):8d}")
# the select side of the same launch (select_descend / select_leaf stamps, g_stamps[0])
lib.bk_debug_stamps.argtypes = [ctypes.c_void_p]
sb = np.zeros((2, 4096, 8), dtype=np.uint64)
assert lib.bk_debug_stamps(sb.ctypes.data_as(ctypes.c_void_p)) == 0
s0 = sb[0, :256, :6].astype(np.int64)
ds = np.diff(s0, axis=1)
for i, n in enumerate(["load", "descent", "build_mask", "mask+state store", "obs write"]):
    print(f"  select: {n:16s} median {int(np.median(ds[:, i])):8d}  max {int(ds[:, i].max()):8d}")
