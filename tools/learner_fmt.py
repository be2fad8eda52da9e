"""Diagnostic: the learner's ResNet-5x64 fwd + bwd + Adam step time at batch B (random inputs,
a plain sum loss: the conv stack is what is timed) in NCHW vs channels_last, with and without
torch.backends.cudnn.benchmark (MIOpen find mode). Usage: python tools/learner_fmt.py [B]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from blokus_rl_amd.nets import ResNet  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
out = {}
for cl in (False, True):
    for bench in (False, True):
        torch.backends.cudnn.benchmark = bench
        torch.manual_seed(0)
        net = ResNet(20, 4, 30433, 5).cuda().train()
        x = torch.randn(B, 8, 20, 20, device="cuda")
        if cl:
            net = net.to(memory_format=torch.channels_last)
            x = x.contiguous(memory_format=torch.channels_last)
        opt = torch.optim.Adam(net.parameters(), lr=1e-3)

        def step():
            p, v = net(x)
            loss = p.float().mean() + v.float().mean()
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()

        for _ in range(5):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        out[f"channels_last={cl},benchmark={bench}"] = round((time.perf_counter() - t0) / 20 * 1e3, 2)
        print(json.dumps(out), flush=True)
