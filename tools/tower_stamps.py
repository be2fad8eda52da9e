"""Per-wave phase times of k_tower_wino from the diagnostics build (make -C blokus_rl_amd/csrc
stamps -> _lib/exp/libst.so): BK_LIB=blokus_rl_amd/_lib/exp/libst.so python tools/tower_stamps.py.
s_memtime stamps per wave (256 boards, 10 layers): 0 kernel start, 1 layer 2 start, 2 after its
prologue barrier, per group g 3+2g MFMA loop done / 4+2g after the group barrier, 29 end; 30/31
s_memrealtime at start/end (in-kernel clock)."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from blokus_rl_amd.engine import load_library  # noqa: E402
from blokus_rl_amd.nets import pack_tower, resnet_tower  # noqa: E402

B, N, nb = 256, 20, 5
lib = load_library()
x = torch.relu(torch.randn(B, 64, N, N, device="cuda")).contiguous(memory_format=torch.channels_last)
ws = [torch.randn(64, 64, 3, 3, device="cuda") / 24 for _ in range(2 * nb)]
ut = pack_tower(ws)
bt = torch.zeros(2 * nb * 64, device="cuda")
for _ in range(200):
    resnet_tower(x, ut, bt, 2 * nb)
torch.cuda.synchronize()
lib.bk_wino_stamps_clear()
resnet_tower(x, ut, bt, 2 * nb)
torch.cuda.synchronize()
st = np.zeros(256 * 8 * 32, dtype=np.uint64)
assert lib.bk_wino_stamps(st.ctypes.data_as(ctypes.c_void_p)) == 0
st = st.reshape(256, 8, 32).astype(np.int64)[:, :4]
st = st.reshape(-1, 32)
q = lambda a: {k: float(np.percentile(a, p)) for k, p in (("p10", 10), ("p50", 50), ("p90", 90), ("max", 100))}  # noqa: E731
out = {"kernel_cycles": q(st[:, 29] - st[:, 0]),
       "clock_ghz": q((st[:, 29] - st[:, 0]) / ((st[:, 31] - st[:, 30]) / 100e6) / 1e9),
       "prologue": q(st[:, 1] - st[:, 0]),
       "per_layer_first3": q((st[:, 2] - st[:, 1]) / 3)}
# layer 2 (the third layer): per group g, MFMA loop end (10 + g) and end after the barrier (3 + g)
prev = st[:, 3 + 6 - 7] if False else None
for g in range(7):
    start = st[:, 3 + g - 1] if g > 0 else None
    if g > 0:
        out[f"L2g{g}_mfma"] = q(st[:, 10 + g] - st[:, 3 + g - 1])
    out[f"L2g{g}_epi"] = q(st[:, 3 + g] - st[:, 10 + g])
print(json.dumps({k: (v["p50"], v["max"]) for k, v in out.items()}))
