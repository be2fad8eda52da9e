"""Debug: bk_leafnet_x3 with nlayers = 1..4 against an fp64 torch emulation of the same layer
chain (stem, convs, ReLU on even non-last convs, last conv + x0 + ReLU); prints max relative
errors of the tower output and the heads."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from blokus_rl_amd.engine import _check, _ptr, load_library  # noqa: E402
from blokus_rl_amd.nets import LeafResNet, ResNet  # noqa: E402

torch.manual_seed(0)
N, B = 20, 4
net = ResNet(N, 4, 100, 2).cuda().eval()
mode = sys.argv[1] if len(sys.argv) > 1 else "normal"
with torch.no_grad():
    c0 = net.res_blocks[0][0]
    if mode == "zero":  # conv0 = 0: the tower output is relu(x0 + bn(0)) ~ the stem output
        c0.weight.zero_()
        c0.bias.zero_()
    elif mode == "center":  # conv0 = identity at the centre tap
        c0.weight.zero_()
        c0.bias.zero_()
        for i in range(64):
            c0.weight[i, i, 1, 1] = 1.0
    elif mode == "shift":  # conv0 = identity at tap (0, 0): out(y, x) = in(y - 1, x - 1)
        c0.weight.zero_()
        c0.bias.zero_()
        for i in range(64):
            c0.weight[i, i, 0, 0] = 1.0
print("mode", mode)
leaf = LeafResNet(net, normalize=False, features=True).eval()
f = leaf.f
convs = [c for blk in f.blocks for c in blk]
obs = (torch.rand((B, 8, N, N), device="cuda") < 0.3).float()
lib = load_library()
print("bounds", leaf.x3_bounds.tolist())
print("sstem", leaf.x3_sstem[:4].tolist(), "stower", leaf.x3_stower[:4].tolist())
for nl in ((1,) if mode != 'normal' else (1, 2, 3, 4)):
    P = 4
    pf = torch.empty((B, 2 * N * N), device="cuda")
    v = torch.empty((B, P), device="cuda")
    out = torch.empty((B, 64, N, N), device="cuda", memory_format=torch.channels_last)
    h = leaf.x3_heads
    _check(lib.bk_leafnet_x3(ctypes.c_void_p(obs.data_ptr()), B, N, 8, _ptr(leaf.x3_wstem), _ptr(leaf.x3_sstem),
                             _ptr(h[0]), nl, _ptr(leaf.x3_wtower), _ptr(leaf.x3_stower), _ptr(leaf.b_tower),
                             _ptr(leaf.x3_bounds), *[_ptr(t) for t in h[1:]], P, _ptr(pf), _ptr(v),
                             ctypes.c_void_p(out.data_ptr()), None))
    torch.cuda.synchronize()
    with torch.no_grad():
        x0 = torch.relu(F.conv2d(obs.double(), f.stem.weight.double(), f.stem.bias.double(), padding=1))
        y = x0
        for i in range(nl):
            c = convs[i]
            y = F.conv2d(y, c.weight.double(), c.bias.double(), padding=1)
            if i + 1 == nl:
                y = torch.relu(y + x0)
            elif i % 2 == 0:
                y = torch.relu(y)
    err = float((out.double() - y).abs().max()) / float(y.abs().max())
    print("nlayers", nl, "tower rel err", err, "out max", float(out.abs().max()), "ref max", float(y.abs().max()))
    d = (out.double() - y).abs()
    bad = (d > 1e-3 * float(y.abs().max())).nonzero()
    print("bad entries", bad.shape[0], "of", d.numel())
    if bad.shape[0]:
        chans = torch.unique(bad[:, 1])
        pix = torch.unique(bad[:, 2] * N + bad[:, 3])
        print(" bad channels", chans.tolist()[:64])
        print(" bad pixels", len(pix), pix.tolist()[:40])
