"""Localise a k_leafnet_x3g mismatch against k_leafnet_x3: per conv count (nblocks), the tower
output's differing pixels (as pixel-map groups) and channels."""
import json
import sys

import torch

sys.path.insert(0, ".")
from blokus_rl_amd.nets import LeafResNet, ResNet, leafnet_x3, leafnet_x3g  # noqa: E402

res = {}
for nb in (1, 2, 5):
    torch.manual_seed(0)
    net = ResNet(20, 4, 30433, nb).cuda().eval()
    leaf = LeafResNet(net, normalize=False, features=True).eval()
    obs = (torch.rand((4, 8, 20, 20), device="cuda") < 0.3).float()
    _, _, o1 = leafnet_x3(obs, leaf, want_out=True)
    _, _, o2 = leafnet_x3g(obs, leaf, want_out=True)
    torch.cuda.synchronize()
    d = (o1 - o2).abs().permute(0, 2, 3, 1).reshape(4, 400, 64)  # [b][pixel][channel]
    bad = d > 0
    px = bad.any(dim=2).any(dim=0).nonzero().flatten().tolist()
    ch = bad.any(dim=1).any(dim=0).nonzero().flatten().tolist()
    res[nb] = {"max": float(d.max()), "bad_pixels": len(px), "first_pixels": px[:40], "bad_channels": ch,
               "boards_bad": bad.any(dim=2).any(dim=1).tolist()}
print(json.dumps(res))
