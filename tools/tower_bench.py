"""bk_resnet_tower (the fused residual tower, one launch) vs the per-layer bk_conv3x3 chain at the
self-play shape (256 boards, 20x20, 5 blocks = 10 convs, fp32): time per tower with HIP events on
the launch stream. Usage: python tools/tower_bench.py [reps] [batch] [blocks]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from blokus_rl_amd.nets import conv3x3, pack_conv3x3, pack_tower, resnet_tower  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
nb = int(sys.argv[3]) if len(sys.argv) > 3 else 5
N = 20
x = torch.relu(torch.randn(B, 64, N, N, device="cuda")).contiguous(memory_format=torch.channels_last)
ws = [torch.randn(64, 64, 3, 3, device="cuda") / 24 for _ in range(2 * nb)]
bs = [torch.randn(64, device="cuda") * 0.1 for _ in range(2 * nb)]
wp = [pack_conv3x3(w) for w in ws]
ut, bt = pack_tower(ws), torch.cat(bs).contiguous()


def chain():
    h = x
    for i in range(2 * nb):
        last = i + 1 == 2 * nb
        h = conv3x3(h, wp[i], bs[i], last or i % 2 == 0, x if last else None)
    return h


def fused():
    return resnet_tower(x, ut, bt, 2 * nb)


res = {"batch": B, "blocks": nb}
st = torch.cuda.current_stream()
for name, fn in (("per_layer", chain), ("fused", fused)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    res[name + "_us"] = e0.elapsed_time(e1) / reps * 1e3
flop = 2.0 * B * N * N * 64 * 9 * 64 * 2 * nb
res["fused_direct_equiv_tflops"] = flop / res["fused_us"] / 1e6
print(json.dumps(res))
