"""k_vec_step7 phase cycles (diagnostic build: tools/build_lib_variant.sh vecst -DBK_VEC_STAMP, then
BK_LIB=blokus_rl_amd/_lib/exp/libvecst.so): per wave, s_memtime at 0 start, 1 state loaded + the
agent's legal origins, 2 agent placed + advance, 3 opponent moves done, 4 the agent's final legal
origins, 5 stores + LDS staging, 6 after the barrier, 7 end. Medians / max over the waves of the
last of a few steps of the 8192-env bench shape."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from blokus_rl_amd.engine import load_library  # noqa: E402
from blokus_rl_amd.vector_env import BlokusVectorEnv  # noqa: E402

E = 8192
env = BlokusVectorEnv(E, 7, 4)
env.reset(seed=0)
for _ in range(30):
    env.step(None)
torch.cuda.synchronize()
lib = load_library()
lib.bk_vec_stamps.argtypes = [ctypes.c_void_p]
s = np.zeros((4096, 8), dtype=np.uint64)
assert lib.bk_vec_stamps(s.ctypes.data_as(ctypes.c_void_p)) == 0
G = int(os.environ.get("BK_VEC_LANES", "16"))
nw = E * G // 64
a = s[:nw].astype(np.int64)
rel = a - a[:, :1]
out = {"waves": nw, "launch_span": int(a[:, 7].max() - a[:, 0].min()), "start_spread": int(a[:, 0].max() - a[:, 0].min())}
for i, nm in enumerate(["", "agent legal", "agent placed", "opponent done", "final legal", "staged", "barrier", "end"]):
    if i:
        d = rel[:, i] - rel[:, i - 1]
        out[nm] = {"median": int(np.median(d)), "max": int(d.max())}
out["total"] = {"median": int(np.median(rel[:, 7])), "max": int(rel[:, 7].max())}
print(json.dumps(out))
