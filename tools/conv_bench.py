"""bk_conv3x3 alone at the self-play shape (256 x 64 x 20 x 20, fp32): time per launch with HIP
events on the launch stream, achieved TFLOP/s vs the 157.3 TF f32 MFMA peak. Usage:
python tools/conv_bench.py [reps] [cin] [batch]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from blokus_rl_amd.nets import conv3x3, pack_conv3x3  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
cin = int(sys.argv[2]) if len(sys.argv) > 2 else 64
B = int(sys.argv[3]) if len(sys.argv) > 3 else 256
N = 20
x = torch.randn(B, cin, N, N, device="cuda")
x = x.contiguous(memory_format=torch.channels_last) if cin == 64 else x.contiguous()
w = pack_conv3x3(torch.randn(64, cin, 3, 3, device="cuda") * 0.05)
b = torch.zeros(64, device="cuda")
for _ in range(5):
    conv3x3(x, w, b, True)
torch.cuda.synchronize()
st = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range(reps):
    conv3x3(x, w, b, True)
e1.record(st)
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / reps * 1e3
flop = 2.0 * B * N * N * 64 * 9 * cin
print(json.dumps({"cin": cin, "batch": B, "us": us, "tflops": flop / us / 1e6, "frac_of_157": flop / us / 1e6 / 157.3}))
