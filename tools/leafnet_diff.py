"""Where a k_leafnet_x3 build goes wrong: the tower output (want_out) against the fp64 forward of
tests/test_leafnet_gpu.py's first case, its error split by channel block of 16 (= the wave that
owns it) and by board. Usage: BK_LIB=... python tools/leafnet_diff.py [B N nblocks]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

from test_leafnet_gpu import _net, _ref64  # noqa: E402

from blokus_rl_amd.nets import LeafResNet, leafnet_x3  # noqa: E402

B, N, nb = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (256, 20, 5)))
net = _net(N, nb, seed=B + N + nb)
g = torch.Generator(device="cuda").manual_seed(B * 3 + N)
obs = (torch.rand((B, 8, N, N), device="cuda", generator=g) < 0.3).float()
leaf = LeafResNet(net, normalize=False, features=True).eval()
pf, v, out = leafnet_x3(obs, leaf, want_out=True)
torch.cuda.synchronize()
_, _, xt = _ref64(net, obs)
err = (out.double() - xt).abs()  # [B, 64, N, N]
scale = float(xt.abs().max())
print("rel max", float(err.max()) / scale)
print("by channel block:", [round(float(err[:, 16 * w:16 * w + 16].max()) / scale, 9) for w in range(4)])
bad = (err.amax(dim=(1, 2, 3)) / scale > 1e-5).nonzero().flatten().tolist()
print("bad boards", len(bad), bad[:20])
if bad:
    e = err[bad[0]].amax(dim=0)  # [N, N]
    print("board", bad[0], "bad pixels", int((e / scale > 1e-5).sum()), "of", N * N)
    # the kernel's pixel map (leafnet.hip LnPixMap): pixel -> (group, column)
    RS = 18 if N == 14 else N + 2
    NG = ((N * N + 15) // 16 + 4) // 5 * 5
    used = [False] * (N * N)
    slot = [-1] * (NG * 16)
    for gi in range(NG):
        for r in range(16):
            for p in range(N * N):
                sl = (p // N + 1) * RS + p % N + 1
                if not used[p] and sl % 16 == r:
                    used[p] = True
                    slot[gi * 16 + r] = sl
                    break
    p = 0
    for i in range(NG * 16):
        if slot[i] >= 0:
            continue
        while p < N * N and used[p]:
            p += 1
        if p == N * N:
            break
        used[p] = True
        slot[i] = (p // N + 1) * RS + p % N + 1
    where = {}
    for i, sl in enumerate(slot):
        if sl >= 0:
            where[(sl // RS - 1) * N + sl % RS - 1] = (i // 16, i % 16)
    for bb in bad[:3]:
        e = err[bb] / scale  # [64, N, N]
        pix = (e.amax(dim=0).flatten() > 1e-5).nonzero().flatten().tolist()
        print("board", bb, [(q, where.get(q), [c for c in range(64) if float(e[c].flatten()[q]) > 1e-5][:6]) for q in pix])
