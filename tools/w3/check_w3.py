"""Quick k_leafnet_w3 check against k_leafnet_x3 (same library, BK_LIB selects it): max relative
difference of the tower outputs and policy features at 256 boards, and the w3 time per launch."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from blokus_rl_amd.nets import LeafResNet, ResNet, leafnet_w3, leafnet_x3  # noqa: E402

torch.manual_seed(0)
net = ResNet(20, 4, 30433, 5).cuda().eval()
leaf = LeafResNet(net, normalize=False, features=True).eval()
obs = (torch.rand((256, 8, 20, 20), device="cuda") < 0.3).float()
pfx, vx, ox = leafnet_x3(obs, leaf, want_out=True)
pfw, vw, ow = leafnet_w3(obs, leaf, want_out=True)
torch.cuda.synchronize()
d = (ow - ox).abs()
bad = torch.nonzero(d.amax(dim=(1, 2, 3)) > 1e-4 * ox.abs().max()).view(-1).tolist()
st = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(10):
    leafnet_w3(obs, leaf)
e0.record(st)
for _ in range(50):
    leafnet_w3(obs, leaf)
e1.record(st)
torch.cuda.synchronize()
print(json.dumps({"lib": os.environ.get("BK_LIB", "default"), "tower_rel": float(d.max() / ox.abs().max()),
                  "pf_rel": float((pfw - pfx).abs().max() / pfx.abs().max()), "boards_bad": len(bad),
                  "first_bad": bad[:5], "us_w3": e0.elapsed_time(e1) / 50 * 1e3}))
