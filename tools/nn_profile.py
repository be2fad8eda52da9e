"""Replay the leaf evaluator's graph (LeafResNet, fp32, batch 256) N times — for rocprofv3."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from blokus_rl_amd.engine import Engine  # noqa: E402
from blokus_rl_amd.alphazero.selfplay import LeafEvaluator  # noqa: E402
from blokus_rl_amd.nets import ResNet  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
eng = Engine(20, 4, 5)
torch.manual_seed(0)
ev = LeafEvaluator(ResNet(20, 4, eng.A, 5).cuda(), eng, 256)
obs = (torch.rand(256, 8, 20, 20, device="cuda") < 0.3).float()
for _ in range(n):
    ev(obs)
torch.cuda.synchronize()
print("ok")
