"""Time bk_leafnet_wx3 vs bk_leafnet_x3 at the leaf batch (B=256, ResNet-5x64, 20x20): HIP events
around each launch on the launch stream; prints one JSON line."""
import json
import sys

import torch

sys.path.insert(0, ".")
from blokus_rl_amd.nets import LeafResNet, ResNet, leafnet_wx3, leafnet_x3  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else 50
torch.manual_seed(0)
net = ResNet(20, 4, 30433, 5).cuda().eval()
leaf = LeafResNet(net, normalize=False, features=True).eval()
obs = (torch.rand((B, 8, 20, 20), device="cuda") < 0.3).float()
st = torch.cuda.current_stream()
out = {}
for name, fn in (("x3", leafnet_x3), ("wx3", leafnet_wx3)):
    for _ in range(5):
        fn(obs, leaf)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(st)
        fn(obs, leaf)
        b.record(st)
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    out[name] = {"us_median": ts[len(ts) // 2], "us_min": ts[0]}
pf1, v1 = leafnet_x3(obs, leaf)
pf2, v2 = leafnet_wx3(obs, leaf)
out["max_abs_diff_pf"] = float((pf1 - pf2).abs().max())
out["max_abs_diff_v"] = float((v1 - v2).abs().max())
print(json.dumps(out))

if "--stamps" in sys.argv:
    import ctypes

    import numpy as np

    from blokus_rl_amd.engine import load_library

    lib = load_library()
    lib.bk_wx_stamps.argtypes = [ctypes.c_void_p]
    leafnet_wx3(obs, leaf)
    torch.cuda.synchronize()
    s = np.zeros(256 * 4 * 64, dtype=np.uint64)
    assert lib.bk_wx_stamps(s.ctypes.data_as(ctypes.c_void_p)) == 0
    s = s.reshape(256, 4, 64).astype(np.int64)[:B]
    rel = s - s[:, :, 0:1]
    med = lambda x: float(np.median(x))  # noqa: E731
    grp = []
    for tg in range(7):
        a, w, y = 2 + 3 * tg, 3 + 3 * tg, 4 + 3 * tg
        prev = rel[:, :, 1] if tg == 0 else rel[:, :, 1 + 3 * tg]
        grp.append({"phaseA": med(rel[:, :, a] - prev) if tg else None, "barrier+R": med(rel[:, :, w] - rel[:, :, a]),
                    "phaseB": med(rel[:, :, y] - rel[:, :, w])})
    res = {"prologue": med(rel[:, :, 1]), "layer1_groups": grp, "layer1": med(rel[:, :, 30] - rel[:, :, 2] + (rel[:, :, 5] - rel[:, :, 4])),
           "total": med(rel[:, :, 31])}
    print(json.dumps(res))
