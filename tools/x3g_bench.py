"""Time bk_leafnet_x3g vs bk_leafnet_x3 at the leaf batch (B=256, ResNet-5x64, 20x20): HIP events
around each launch on the launch stream; checks the tower output bitwise; prints one JSON line."""
import json
import sys

import torch

sys.path.insert(0, ".")
from blokus_rl_amd.nets import LeafResNet, ResNet, leafnet_x3, leafnet_x3g  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
B = int(args[0]) if args else 256
reps = int(args[1]) if len(args) > 1 else 50
torch.manual_seed(0)
net = ResNet(20, 4, 30433, 5).cuda().eval()
leaf = LeafResNet(net, normalize=False, features=True).eval()
obs = (torch.rand((B, 8, 20, 20), device="cuda") < 0.3).float()
st = torch.cuda.current_stream()
out = {}
_, _, o1 = leafnet_x3(obs, leaf, want_out=True)
_, _, o2 = leafnet_x3g(obs, leaf, want_out=True)
torch.cuda.synchronize()
out["tower_bitwise"] = bool(torch.equal(o1, o2))
out["tower_max_rel_diff"] = float((o1 - o2).abs().max() / o1.abs().max())
out["tower_max_abs_diff"] = float((o1 - o2).abs().max())
for name, fn in (("x3", leafnet_x3), ("x3g", leafnet_x3g)) * 2:
    for _ in range(5):
        fn(obs, leaf)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(st)
        fn(obs, leaf)
        b.record(st)
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    out[name] = {"us_median": round(ts[len(ts) // 2], 1), "us_min": round(ts[0], 1)}
pf1, v1 = leafnet_x3(obs, leaf)
pf2, v2 = leafnet_x3g(obs, leaf)
out["max_abs_diff_pf"] = float((pf1 - pf2).abs().max())
out["max_abs_diff_v"] = float((v1 - v2).abs().max())
print(json.dumps(out))

if "--stamps" in sys.argv:
    import ctypes

    import numpy as np

    from blokus_rl_amd.engine import load_library

    lib = load_library()
    lib.bk_x3g_stamps.argtypes = [ctypes.c_void_p]
    leafnet_x3g(obs, leaf)
    torch.cuda.synchronize()
    s = np.zeros(256 * 4 * 16, dtype=np.uint64)
    assert lib.bk_x3g_stamps(s.ctypes.data_as(ctypes.c_void_p)) == 0
    s = s.reshape(256, 4, 16).astype(np.int64)[:B, :, :10]
    d = np.diff(s, axis=2)  # [block][wave][chunk]: cycles of chunk c (its reads, MFMAs, extras)
    print(json.dumps({"chunk_cycles_median": [float(np.median(d[:, :, c])) for c in range(d.shape[2])],
                      "step_cycles_median": float(np.median(s[:, :, 9] - s[:, :, 0])),
                      "step_cycles_by_wave": [float(np.median(s[:, w, 9] - s[:, w, 0])) for w in range(4)]}))
    lib.bk_x3g_steps.argtypes = [ctypes.c_void_p]
    s2 = np.zeros(256 * 4 * 64, dtype=np.uint64)
    assert lib.bk_x3g_steps(s2.ctypes.data_as(ctypes.c_void_p)) == 0
    s2 = s2.reshape(256, 4, 64).astype(np.int64)[:B, :, :50]
    d2 = np.diff(s2, axis=2)
    print(json.dumps({"step_cycles_conv1_2": [float(np.median(d2[:, :, k])) for k in range(d2.shape[2])]}))
