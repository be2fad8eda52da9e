"""Diagnostic: per-tree phase cycles of k_leaf_step_ov (BK_STAMPS build,
BK_LIB=blokus_rl_amd/_lib/diag/libblokus_hip_diag.so) in the last launch of a few self-play plies
(bench config): the critical path of the slowest trees and its relation to the leaf's K."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from blokus_rl_amd import engine  # noqa: E402
from blokus_rl_amd.alphazero.selfplay import SelfPlay  # noqa: E402
from blokus_rl_amd.engine import Engine  # noqa: E402
from blokus_rl_amd.nets import build_model  # noqa: E402

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
lib.bk_debug_stamps.argtypes = [ctypes.c_void_p]
sb = np.zeros((2, 4096, 8), dtype=np.uint64)
assert lib.bk_debug_stamps(sb.ctypes.data_as(ctypes.c_void_p)) == 0
a = buf[:256].astype(np.int64)
g0, g1 = sb[0, :256].astype(np.int64), sb[1, :256].astype(np.int64)
ok = (a[:, 7] > 0) & (a[:, 4] > 0)
a, g0, g1 = a[ok], g0[ok], g1[ok]
rel = a - a[:, :1]
names = ["node added (wave 1)", "wave0 backup", "wave0 descent", "logits (last wave)", "children", "mask done", "obs/end"]
out = {"trees": int(ok.sum()), "total_median": float(np.median(rel[:, 7])), "total_max": float(rel[:, 7].max()),
       "start_spread": float(a[:, 0].max() - a[:, 0].min())}
for i, nm in zip([1, 2, 3, 4, 5, 6, 7], names):
    out[nm] = {"median": float(np.median(rel[:, i])), "p90": float(np.percentile(rel[:, i], 90)),
               "max": float(rel[:, i].max())}
extra = {"children stores issued": a[:, 9] - a[:, 0], "wave0 out of mask claims": a[:, 8] - a[:, 0], "select_leaf stores issued": g0[:, 4] - a[:, 0],
         "select_leaf obs issued": g0[:, 5] - a[:, 0], "descent probe (sum)": g0[:, 6], "descent PUCT scan (sum)": g0[:, 7],
         "descent placement (sum)": g1[:, 7], "descent next-mover check (sum)": g1[:, 6]}
for nm, v in extra.items():
    out[nm] = {"median": float(np.median(v)), "p90": float(np.percentile(v, 90)), "max": float(v.max())}
# the leaf bitmask claims per (tree, wave): entry / exit relative to the tree's start, slices, longest slice
lib.bk_debug_mask_stamps.argtypes = [ctypes.c_void_p]
ms = np.zeros((256, 16, 6), dtype=np.uint64)
if lib.bk_debug_mask_stamps(ms.ctypes.data_as(ctypes.c_void_p)) == 0:
    ms = ms[ok].astype(np.int64)
    t0 = a[:, :1]
    ent, ex = ms[:, :, 0] - t0, ms[:, :, 2] - t0
    out["mask claims"] = {"entry_median_per_wave": np.median(ent, axis=0).tolist(),
                          "exit_median_per_wave": np.median(ex, axis=0).tolist(),
                          "slices_mean_per_wave": ms[:, :, 1].mean(axis=0).round(2).tolist(),
                          "longest_slice_median": float(np.median(ms[:, :, 3].max(axis=1))),
                          "slice_median_of_claiming_waves": float(np.median(ms[:, :, 3][ms[:, :, 1] > 0])),
                          "warm_slice_median": float(np.median(ms[:, :, 4][ms[:, :, 1] > 0])),
                          "row_ctx_median": float(np.median((ms[:, :, 5] - ms[:, :, 0])[ms[:, :, 1] > 0]))}
slow = np.argsort(rel[:, 7])[-10:]
out["slowest10"] = [[int(x) for x in rel[j, 1:]] for j in slow]
K = sp.mcts.__dict__.get("_k", None)
print(json.dumps(out))
