"""A/B check of two builds of bk_leafnet_x3: `dump OUT.pt` runs the kernel of the library BK_LIB
points at (default: the in-tree build) on seeded nets and observations (20x20 and 14x14) and saves
the outputs; `cmp A.pt B.pt` reports whether two dumps are bitwise equal (exit 1 if not).
Usage: BK_LIB=... python tools/leafnet_ab.py dump gpurun_out/a.pt; python tools/leafnet_ab.py cmp a.pt b.pt"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def dump(path):
    from blokus_rl_amd.nets import LeafResNet, ResNet, leafnet_x3

    res = {}
    for N, P, B, blocks in ((20, 4, 64, 5), (14, 4, 24, 2)):
        torch.manual_seed(N)
        net = ResNet(N, P, 100, blocks).cuda().eval()
        with torch.no_grad():  # non-trivial folded BN
            for m in net.modules():
                if isinstance(m, torch.nn.BatchNorm2d):
                    m.running_mean.uniform_(-0.2, 0.2)
                    m.running_var.uniform_(0.5, 1.5)
                    m.weight.uniform_(0.5, 1.5)
                    m.bias.uniform_(-0.2, 0.2)
        leaf = LeafResNet(net, normalize=False, features=True).eval()
        obs = (torch.rand((B, 8, N, N), device="cuda") < 0.3).float()
        pf, v, out = leafnet_x3(obs, leaf, want_out=True)
        torch.cuda.synchronize()
        res[N] = (pf.cpu(), v.cpu(), out.contiguous().cpu())
    torch.save(res, path)
    print("dumped", path)


def cmp(a, b):
    ra, rb = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    ok = True
    for N in ra:
        for name, x, y in zip(("pf", "v", "out"), ra[N], rb[N]):
            same = torch.equal(x, y)
            diff = float((x.double() - y.double()).abs().max())
            print(f"N={N} {name}: bitwise {'equal' if same else 'DIFFERENT'} (max |diff| {diff:.3g})")
            ok &= same
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
