"""Diagnostic for bk_leafnet_wx3: the tower output vs an fp64 forward, error located by tile group,
tile, pixel-in-tile and channel (prints a summary)."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_leafnet_gpu import _net, _ref64  # noqa: E402

from blokus_rl_amd.nets import LeafResNet, leafnet_wx3  # noqa: E402

nblocks = int(sys.argv[1]) if len(sys.argv) > 1 else 1
B = 4
net = _net(20, nblocks, seed=5)
g = torch.Generator(device="cuda").manual_seed(1)
obs = torch.randn((B, 8, 20, 20), device="cuda", generator=g)
leaf = LeafResNet(net, normalize=False, features=True).eval()
pf, v, out = leafnet_wx3(obs, leaf, want_out=True)
torch.cuda.synchronize()
_, _, xt = _ref64(net, obs)
err = (out.double() - xt).abs()  # [B, 64, 20, 20]
scale = float(xt.abs().max())
print("max rel err", float(err.max()) / scale)
e = err.amax(dim=0) / scale  # [64, 20, 20]
tile_err = e.view(64, 10, 2, 10, 2).amax(dim=(0, 2, 4))  # [10, 10]
print("per tile (x1e6):")
for r in range(10):
    print(" ".join(f"{float(x) * 1e6:8.1f}" for x in tile_err[r]))
print("per pixel-in-tile:", [float(e.view(64, 10, 2, 10, 2)[:, :, a, :, b].max()) for a in range(2) for b in range(2)])
ch = e.amax(dim=(1, 2))
print("per channel quad:", [round(float(ch[4 * k:4 * k + 4].max()) * 1e6, 1) for k in range(16)])
print("batch:", [float(err[i].max()) / scale for i in range(B)])
