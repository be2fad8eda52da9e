"""Config-5 kernels for a rocprofv3 PMC pass (tools/gpu/pmc_kernel.sh): eager launches of one
mode at the benchmark size, after a warm-up. mode: random (k_vec_step7 with in-kernel agent
draws: the bench headline's kernel), policy (the fused draw + step, k_vec_step7<4, 16, 2>, random
[E, A] logits resident in HBM) or draw (the standalone k_vec_policy, then the step with its ids).  usage: python tools/vec_pmc.py <mode> [steps] [envs]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from blokus_rl_amd.vector_env import BlokusVectorEnv  # noqa: E402

mode = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
E = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
env = BlokusVectorEnv(E, 7, 4)
env.reset(seed=0)
logits = (torch.randn((E, env.eng.A), device=env.device) * 2.0).contiguous()
for i in range(20 + steps):
    if mode == "random":
        env.step_raw(None)
    elif mode == "policy":
        env.step_policy(logits)
    else:
        env.step_policy(logits, fused=False)
torch.cuda.synchronize()
print(mode, steps, "steps ok")
