"""k_leafnet_x3p phase stamps (diagnostic build, `make -C blokus_rl_amd/csrc lnstamps`, run with
BK_LIB=blokus_rl_amd/_lib/exp/liblnst.so): per wave, s_memtime before / after each of the first
15 tower barriers. Prints, per barrier b (P_0 = 0; then X Q R P per conv), the median over the
256 workgroups of each half's work since the previous barrier and its wait at b (cycles).
Usage: BK_LIB=... python tools/lnp_stamps.py [batch]"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from blokus_rl_amd.engine import load_library  # noqa: E402
from blokus_rl_amd.nets import LeafResNet, ResNet, leafnet_x3  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
torch.manual_seed(0)
net = ResNet(20, 4, 30433, 5).cuda().eval()
leaf = LeafResNet(net, normalize=False, features=True).eval()
obs = (torch.rand((B, 8, 20, 20), device="cuda") < 0.3).float()
for _ in range(50):
    leafnet_x3(obs, leaf)
torch.cuda.synchronize()
lib = load_library()
lib.bk_lnp_stamps.argtypes = [ctypes.c_void_p]
s = np.zeros(256 * 8 * 32, dtype=np.uint64)
assert lib.bk_lnp_stamps(s.ctypes.data_as(ctypes.c_void_p)) == 0
s = s.reshape(256, 8, 32).astype(np.int64)[:B]
names = ["P0", "X-1", "Q0", "R0", "P1", "X0", "Q1", "R1", "P2", "X1", "Q2", "R2", "P3", "X2", "Q3"]
rows = []
for b in range(1, 15):
    row = {"barrier": names[b]}
    for h, hn in ((0, "top"), (1, "bottom")):
        w = s[:, 4 * h:4 * h + 4]
        work = w[:, :, 2 * b] - w[:, :, 2 * b - 1]
        wait = w[:, :, 2 * b + 1] - w[:, :, 2 * b]
        row[hn + "_work"] = int(np.median(work))
        row[hn + "_wait"] = int(np.median(wait))
    rows.append(row)
    print(json.dumps(row))
tot = s[:, :, 31] - s[:, :, 30]
print(json.dumps({"kernel_cycles_median": int(np.median(tot)), "layer_cycles_P1_to_P2": int(np.median(s[:, :, 17] - s[:, :, 9])),
                  "layer_cycles_P2_to_P3": int(np.median(s[:, :, 25] - s[:, :, 17]))}))
