"""Probe: the learner's policy Linear (800 -> 30433, batch 1024) as fp32 GEMMs (hipBLASLt) vs the
split-f16 x3 form (hi*hi + lo*hi + hi*lo with f32 accumulation) as ONE f16 GEMM with the three
products concatenated along K (torch.mm(..., out_dtype=float32)); time and error vs fp64."""
import time

import torch

dev = "cuda"
torch.manual_seed(0)
B, F, A = 1024, 800, 30433
pf = torch.relu(torch.randn(B, F, device=dev))
W = torch.randn(A, F, device=dev) * 0.02
gl = torch.randn(B, A, device=dev) * 1e-6


def split(x, s):
    xs = x * s
    hi = xs.half()
    lo = (xs - hi.float()).half()
    return hi, lo


def pow2_scale(x, target=2.0 ** 12):
    m = float(x.abs().max())
    return 2.0 ** (int(torch.floor(torch.log2(torch.tensor(target / m)))) if m > 0 else 0)


def t(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        y = fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n, y


def x3_mm(a, b):  # a [M,K] f32, b [K,N] f32 -> f32 [M,N]
    sa, sb = pow2_scale(a), pow2_scale(b)
    ah, al = split(a, sa)
    bh, bl = split(b, sb)
    A3 = torch.cat([ah, al, ah], dim=1)
    B3 = torch.cat([bh, bh, bl], dim=0)
    return torch.mm(A3, B3, out_dtype=torch.float32) * (1.0 / (sa * sb))


for name, a, b in (("fwd pf.W^T", pf, W.t()), ("dgrad gl.W", gl, W), ("wgrad gl^T.pf", gl.t(), pf)):
    ref = (a.double() @ b.double())
    bound = a.abs().double() @ b.abs().double()
    ms32, y32 = t(lambda: a @ b)
    ms3, y3 = t(lambda: x3_mm(a, b))
    a16, b16 = a.half().contiguous(), b.half().contiguous()
    msh, _ = t(lambda: torch.mm(a16, b16, out_dtype=torch.float32))
    e32 = float(((y32.double() - ref).abs() / (bound + 1e-300)).max())
    e3 = float(((y3.double() - ref).abs() / (bound + 1e-300)).max())
    print(f"{name}: fp32 {ms32:.3f} ms (err/bound {e32:.2e}) | x3 {ms3:.3f} ms (err/bound {e3:.2e}) | one f16 GEMM {msh:.3f} ms", flush=True)
