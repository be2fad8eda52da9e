"""Per-wave phase times of the Winograd conv kernels from the diagnostics build
(make -C blokus_rl_amd/csrc stamps -> _lib/exp/libst.so, -DBK_WINO_STAMP=1):
BK_LIB=blokus_rl_amd/_lib/exp/libst.so [BK_CONV_WINO=1] python tools/wino_stamps.py [batch].
Stamps are s_memtime (shader clock) per wave. Form 1 (k_conv3x3_wino, 8 waves): 0 start, 1 after
the U fill, per task t: 2+3t loop start, 3+3t MFMA loop issued, 4+3t epilogue done. Form 2
(k_conv3x3_wino2, 4 waves): 0 start, 1 after the prologue barrier, per group r: 2+3r loop top,
3+3r MFMA loop done, 4+3r after the group barrier; 29 end; 30/31 s_memrealtime (100 MHz) at
start/end, giving the in-kernel clock."""
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
form2 = os.environ.get("BK_CONV_WINO", "2") != "1"
lib = load_library()
x = torch.relu(torch.randn(B, 64, 20, 20, device="cuda")).contiguous(memory_format=torch.channels_last)
w = pack_conv3x3(torch.randn(64, 64, 3, 3, device="cuda") * 0.05)
b = torch.zeros(64, device="cuda")
for _ in range(2000):  # >= 2 s of back-to-back launches so the clock settles
    conv3x3(x, w, b, True)
torch.cuda.synchronize()
lib.bk_wino_stamps_clear()
conv3x3(x, w, b, True)
torch.cuda.synchronize()
st = np.zeros(256 * 8 * 32, dtype=np.uint64)
assert lib.bk_wino_stamps(st.ctypes.data_as(ctypes.c_void_p)) == 0
st = st.reshape(256, 8, 32).astype(np.int64)
nw = 4 if form2 else 8
live = st[:, :nw, 0] > 0
fill = (st[:, :nw, 1] - st[:, :nw, 0])[live]
loops, epis, gaps, ntask, ends, clocks = [], [], [], [], [], []
t_first = st[:, :nw, 0][live].min()
for blk in range(256):
    for wv in range(nw):
        if not live[blk, wv]:
            continue
        s = st[blk, wv]
        t = 0
        while 4 + 3 * t < 29 and s[4 + 3 * t] > 0:
            loops.append(s[3 + 3 * t] - s[2 + 3 * t])
            epis.append(s[4 + 3 * t] - s[3 + 3 * t])
            if t > 0:
                gaps.append(s[2 + 3 * t] - s[4 + 3 * t - 3])
            t += 1
        ntask.append(t)
        ends.append(s[:29][s[:29] > 0].max() - s[0])
        if form2 and s[31] > s[30]:
            clocks.append((s[29] - s[0]) / ((s[31] - s[30]) / 100e6) / 1e9)
q = lambda a: {k: float(np.percentile(a, p)) for k, p in (("p10", 10), ("p50", 50), ("p90", 90), ("max", 100))} if len(a) else None  # noqa: E731
out = {"form": 2 if form2 else 1, "batch": B, "waves": int(live.sum()), "prologue": q(fill), "mfma_loop": q(loops),
       "epilogue_barrier": q(epis), "gap": q(gaps), "groups": q(ntask), "wave_life": q(ends),
       "start_skew": q((st[:, :nw, 0][live] - t_first)), "clock_ghz": q(clocks)}
if form2:
    # group index 2 by quarters of its k-steps (stamps 8 = start, 23/24/25 = steps 4/8/12, 9 = end)
    g2 = st[:, :nw][live]
    g2 = g2[(g2[:, 9] > 0) & (g2[:, 25] > 0)]
    out["g2_steps_0_3"] = q(g2[:, 23] - g2[:, 8])
    out["g2_steps_4_7"] = q(g2[:, 24] - g2[:, 23])
    out["g2_steps_8_11"] = q(g2[:, 25] - g2[:, 24])
    out["g2_steps_12_15"] = q(g2[:, 9] - g2[:, 25])
    g0 = st[:, :nw][live]
    out["g0_loop"] = q(g0[:, 3] - g0[:, 2])
    out["prologue_first_window"] = q(g0[:, 27] - g0[:, 0])
    out["prologue_transform"] = q(g0[:, 28] - g0[:, 27])
    out["prologue_barrier"] = q(g0[:, 1] - g0[:, 28])
    blk = st[:, :nw, 0]
    ok = (blk > 0).all(axis=1)
    out["block_start_skew"] = q(blk[ok].max(axis=1) - blk[ok].min(axis=1))
print(json.dumps(out, indent=1))
