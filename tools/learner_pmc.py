"""The learner's device path (bench.py's `learner` main leg: batch 1024, channels_last ResNet-5x64,
k_conv_x3 / k_conv_x3_wgrad / trainbn.hip / k_policy_loss(+grad)) for rocprofv3 PMC passes
(tools/gpu/pmc_kernel.sh): warm-up 3 + 10 train steps, then the loss kernels' own timing loop."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blokus_rl_amd.alphazero.learner_bench import bench_learner  # noqa: E402
from blokus_rl_amd.engine import Engine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
r = bench_learner(Engine(20, 4, 5), 1, 0, 1024, steps, 3, rows=8192, device_path="auto")
print("device_path", r["device_path"], "elapsed", r["elapsed_s"])
