"""bk_leafnet_x3 at the self-play shape (256 boards 20x20, ResNet-5x64): time per launch with HIP
events on the launch stream, and (--stamps, with BK_LIB=blokus_rl_amd/_lib/exp/liblnst.so from
`make -C blokus_rl_amd/csrc lnstamps`) the per-wave phase times of one launch from its s_memtime
stamps: 0 start, 1 stem input staged, 2 stem MFMAs done, 3 stem epilogue done, 4+2L / 5+2L layer
L's MFMA loop / epilogue done (L < 8), 20 heads' partials, 29 end; 30/31 s_memrealtime (100 MHz).
Usage: python tools/leafnet_bench.py [reps] [batch] [--stamps]"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from blokus_rl_amd.engine import load_library  # noqa: E402
from blokus_rl_amd.nets import LeafResNet, ResNet, leafnet_x3  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
reps = int(args[0]) if args else 200
B = int(args[1]) if len(args) > 1 else 256
torch.manual_seed(0)
net = ResNet(20, 4, 30433, 5).cuda().eval()
leaf = LeafResNet(net, normalize=False, features=True).eval()
obs = (torch.rand((B, 8, 20, 20), device="cuda") < 0.3).float()
st = torch.cuda.current_stream()
for _ in range(20):
    leafnet_x3(obs, leaf)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range(reps):
    leafnet_x3(obs, leaf)
e1.record(st)
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / reps * 1e3
ng = 25
flop = B * 4 * ng * 3 * (2.0 * 16 * 16 * 32) * (18 * 10 + 3)
res = {"batch": B, "us_per_launch": us, "executed_tflops": flop / us / 1e6, "frac_of_2.5PF": flop / us / 1e6 / 2500}
if "--stamps" in sys.argv:
    lib = load_library()
    lib.bk_ln_stamps_clear.restype = ctypes.c_int
    lib.bk_ln_stamps.argtypes = [ctypes.c_void_p]
    assert lib.bk_ln_stamps_clear() == 0
    leafnet_x3(obs, leaf)
    torch.cuda.synchronize()
    s = np.zeros(256 * 4 * 32, dtype=np.uint64)
    assert lib.bk_ln_stamps(s.ctypes.data_as(ctypes.c_void_p)) == 0
    s = s.reshape(256, 4, 32).astype(np.int64)[:B]
    t0 = s[:, :, 0:1]
    rel = s - t0
    clk = (s[:, :, 29] - s[:, :, 0]) / ((s[:, :, 31] - s[:, :, 30]) / 100e6) / 1e9
    names = {1: "stem_in", 2: "stem_mfma", 3: "stem_epi", 20: "heads_part", 29: "end"}
    for L in range(8):
        names[4 + 2 * L] = f"L{L}_mfma"
        names[5 + 2 * L] = f"L{L}_epi"
    prev = 0
    phases = {}
    for i in sorted(names):
        d = rel[:, :, i] - rel[:, :, prev]
        phases[names[i]] = float(np.median(d))
        prev = i
    res["phase_cycles_median"] = phases
    epi = {}  # layer 1's epilogue: compute, wave max, barrier 1, grid writes, barrier 2
    for i, nm in zip(range(21, 26), ("compute", "wave_max", "barrier1", "write_act", "barrier2")):
        prev_i = 4 + 2 * 1 if i == 21 else i - 1
        epi[nm] = float(np.median(rel[:, :, i] - rel[:, :, prev_i]))
    res["layer1_epilogue_cycles_median"] = epi
    # layer 1's MFMA loop: prime (from layer 0's epilogue end), chunk 0, chunks 1-8, chunks 9-17 + drain
    res["layer1_loop_cycles_median"] = {
        "prime": float(np.median(rel[:, :, 26] - rel[:, :, 5])),
        "chunk0": float(np.median(rel[:, :, 27] - rel[:, :, 26])),
        "chunks1_8": float(np.median(rel[:, :, 28] - rel[:, :, 27])),
        "chunks9_17": float(np.median(rel[:, :, 6] - rel[:, :, 28])),
    }
    res["total_cycles_median"] = float(np.median(rel[:, :, 29]))
    res["clock_ghz_median"] = float(np.median(clk))
    res["mfma_cycles_per_layer_floor"] = 18 * ng * 3 * 16
print(json.dumps(res))
