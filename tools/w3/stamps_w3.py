"""Per-wave phase times of one k_leafnet_w3 launch from its s_memtime stamps (BK_LIB =
blokus_rl_amd/_lib/exp/libw3st.so from `make -C blokus_rl_amd/csrc w3stamps`), 256 boards 20x20,
ResNet-5x64: stem, layer 1 unit by unit (issue time from the barrier to the next barrier, and the
wait at each barrier), the layer end, the tower, the heads; medians over the 1024 waves.
Usage: BK_LIB=... python tools/w3/stamps_w3.py"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from blokus_rl_amd.engine import load_library  # noqa: E402
from blokus_rl_amd.nets import LeafResNet, ResNet, leafnet_w3  # noqa: E402

torch.manual_seed(0)
net = ResNet(20, 4, 30433, 5).cuda().eval()
leaf = LeafResNet(net, normalize=False, features=True).eval()
obs = (torch.rand((256, 8, 20, 20), device="cuda") < 0.3).float()
for _ in range(5):
    leafnet_w3(obs, leaf)
torch.cuda.synchronize()
lib = load_library()
lib.bk_w3_stamps.argtypes = [ctypes.c_void_p]
s = np.zeros(256 * 4 * 128, dtype=np.uint64)
assert lib.bk_w3_stamps(s.ctypes.data_as(ctypes.c_void_p)) == 0
s = s.reshape(256, 4, 128).astype(np.int64)
rel = s - s[:, :, 0:1]
med = lambda x: float(np.median(x))  # noqa: E731
res = {"total": med(rel[:, :, 63]), "stem": med(rel[:, :, 1]), "layer0_and_1_to_start": med(rel[:, :, 2] - rel[:, :, 1]),
       "l1_first_v_and_u_wait": med(rel[:, :, 3] - rel[:, :, 2])}
units = []
for u in range(28):
    before = rel[:, :, 4 + u]
    after = rel[:, :, 32 + u]
    prev_after = rel[:, :, 32 + u - 1] if u else rel[:, :, 3]
    units.append({"u": u, "issue": med(before - prev_after), "barrier_wait": med(after - before)})
res["l1_units"] = units
res["l1_last_unit_and_epilogue"] = med(rel[:, :, 60] - rel[:, :, 59])
res["l1_end_barrier"] = med(rel[:, :, 61] - rel[:, :, 60])
res["l1_total"] = med(rel[:, :, 61] - rel[:, :, 2])
res["tower_end"] = med(rel[:, :, 62])
res["heads"] = med(rel[:, :, 63] - rel[:, :, 62])
res["sum_issue"] = sum(x["issue"] for x in units)
res["sum_barrier"] = sum(x["barrier_wait"] for x in units)
# inside units 9, 10, 12 of layer 1: after the barrier -> V pieces 0-1 -> triple 0..7 -> fetch
for u, base in ((9, 64), (10, 96), (12, 80)):
    marks = [rel[:, :, 32 + u]] + [rel[:, :, base + j] for j in range(12)]
    names = ["write_out+bload0", "pieces01"] + [f"triple{i}+piece" for i in range(8)] + ["tail", "fetch"]
    res[f"unit{u}_inside"] = {nm: med(marks[j + 1] - marks[j]) for j, nm in enumerate(names)}
print(json.dumps(res))
