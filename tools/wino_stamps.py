"""Per-wave phase times of k_conv3x3_wino from the diagnostics build (-DBK_WINO_STAMP=1):
BK_LIB=blokus_rl_amd/_lib/exp/libst.so python tools/wino_stamps.py [batch]. Stamps are s_memtime
(shader clock) per wave: 0 start, 1 after the U fill, then per task 2+3t loop start, 3+3t MFMA
loop issued, 4+3t epilogue done."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from blokus_rl_amd.engine import load_library  # noqa: E402
from blokus_rl_amd.nets import conv3x3, pack_conv3x3  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
lib = load_library()
x = torch.relu(torch.randn(B, 64, 20, 20, device="cuda")).contiguous(memory_format=torch.channels_last)
w = pack_conv3x3(torch.randn(64, 64, 3, 3, device="cuda") * 0.05)
b = torch.zeros(64, device="cuda")
for _ in range(20):
    conv3x3(x, w, b, True)
torch.cuda.synchronize()
lib.bk_wino_stamps_clear()
conv3x3(x, w, b, True)
torch.cuda.synchronize()
st = np.zeros(256 * 8 * 32, dtype=np.uint64)
assert lib.bk_wino_stamps(st.ctypes.data_as(ctypes.c_void_p)) == 0
st = st.reshape(256, 8, 32).astype(np.int64)
live = st[:, :, 0] > 0
t0 = st[:, :, 0][live].min()
fill = (st[:, :, 1] - st[:, :, 0])[live]
loops, epis, gaps, ntask = [], [], [], []
for blk in range(256):
    for wv in range(8):
        if not live[blk, wv]:
            continue
        s = st[blk, wv]
        t = 0
        while 4 + 3 * t < 32 and s[4 + 3 * t] > 0:
            loops.append(s[3 + 3 * t] - s[2 + 3 * t])
            epis.append(s[4 + 3 * t] - s[3 + 3 * t])
            if t > 0:
                gaps.append(s[2 + 3 * t] - s[4 + 3 * t - 3])
            t += 1
        ntask.append(t)
ends = []
for blk in range(256):
    for wv in range(8):
        if live[blk, wv]:
            s = st[blk, wv]
            ends.append(s[s > 0].max() - s[0])
q = lambda a: {k: float(np.percentile(a, p)) for k, p in (("p10", 10), ("p50", 50), ("p90", 90), ("max", 100))} if len(a) else None
print(json.dumps({"batch": B, "waves": int(live.sum()), "fill": q(fill), "loop": q(loops), "epilogue": q(epis),
                  "gap": q(gaps), "tasks": q(ntask), "wave_life": q(ends)}, indent=1))
