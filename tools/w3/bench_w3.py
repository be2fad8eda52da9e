"""k_leafnet_w3 vs k_leafnet_x3 at the self-play shape (256 boards 20x20, ResNet-5x64): time per
launch (HIP events on the launch stream, interleaved A/B rounds) and the distance between the two
kernels' outputs and to an fp64 forward. Usage: python tools/w3/bench_w3.py [reps] [rounds]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from blokus_rl_amd.nets import FusedResNet, LeafResNet, ResNet, leafnet_w3, leafnet_x3  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
B = 256
torch.manual_seed(0)
net = ResNet(20, 4, 30433, 5).cuda().eval()
leaf = LeafResNet(net, normalize=False, features=True).eval()
obs = (torch.rand((B, 8, 20, 20), device="cuda") < 0.3).float()
st = torch.cuda.current_stream()
res = {"batch": B}
pfx, vx, ox = leafnet_x3(obs, leaf, want_out=True)
pfw, vw, ow = leafnet_w3(obs, leaf, want_out=True)
torch.cuda.synchronize()
with torch.no_grad():
    fd = FusedResNet(net).double().eval()
    x = torch.relu(fd.stem(obs.double()))
    h = x
    for c1, c2 in fd.blocks:
        h = c2(torch.relu(c1(h)))
    xt = torch.relu(x + h)
    pf64 = torch.relu(fd.policy_conv(xt)).flatten(1)


def rel(a, r):
    return float((a.double() - r).abs().max()) / float(r.abs().max())


res["rel_err_tower_x3"] = rel(ox, xt)
res["rel_err_tower_w3"] = rel(ow, xt)
res["rel_err_pf_x3"] = rel(pfx, pf64)
res["rel_err_pf_w3"] = rel(pfw, pf64)
res["max_abs_v_w3_minus_x3"] = float((vw - vx).abs().max())
times = {"x3": [], "w3": []}
for _ in range(rounds):
    for name, fn in (("x3", leafnet_x3), ("w3", leafnet_w3)):
        for _ in range(10):
            fn(obs, leaf)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn(obs, leaf)
        e1.record(st)
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / reps * 1e3)
res["us_per_launch"] = times
res["speedup_w3_over_x3"] = min(times["x3"]) / min(times["w3"])
print(json.dumps(res))
