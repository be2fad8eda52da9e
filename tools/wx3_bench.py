"""Time bk_leafnet_wx3 vs bk_leafnet_x3 at the leaf batch (B=256, ResNet-5x64, 20x20): HIP events
around each launch on the launch stream; prints one JSON line."""
import json
import sys

import torch

sys.path.insert(0, ".")
from blokus_rl_amd.nets import LeafResNet, ResNet, leafnet_wx3, leafnet_x3  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
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
