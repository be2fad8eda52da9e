"""k_leafnet_w3 alone at the self-play shape (256 boards, ResNet-5x64), `reps` launches: the
driver of the rocprofv3 passes (tools/gpu/w3pmc.sh). Usage: python tools/w3/run_w3.py [reps] [x3]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from blokus_rl_amd.nets import LeafResNet, ResNet, leafnet_w3, leafnet_x3  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
fn = leafnet_x3 if len(sys.argv) > 2 and sys.argv[2] == "x3" else leafnet_w3
torch.manual_seed(0)
net = ResNet(20, 4, 30433, 5).cuda().eval()
leaf = LeafResNet(net, normalize=False, features=True).eval()
obs = (torch.rand((256, 8, 20, 20), device="cuda") < 0.3).float()
for _ in range(reps):
    fn(obs, leaf)
torch.cuda.synchronize()
