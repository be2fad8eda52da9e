"""A/B bitwise check of two engine builds: a few self-play plies (bench config 3 shape) with the
library BK_LIB names, the roots' visit distributions and the ply's actions saved to argv[1]
(.npz). Run once per build and compare the files with --compare a.npz b.npz."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    same = all(np.array_equal(a[k], b[k]) for k in a.files)
    print("bitwise equal" if same else "DIFFERENT", {k: int((a[k] != b[k]).sum()) for k in a.files})
    sys.exit(0 if same else 1)

import torch  # noqa: E402

from blokus_rl_amd.alphazero.selfplay import SelfPlay  # noqa: E402
from blokus_rl_amd.engine import Engine  # noqa: E402
from blokus_rl_amd.nets import build_model  # noqa: E402

eng = Engine(20, 4, 5)
torch.manual_seed(0)
net = build_model("resnet", 20, 4, eng.A, num_res_blocks=5).to(eng.device).eval()
sp = SelfPlay(eng, net, 256, num_sims=100, seed=77, continuous=True)
out = {}
for i in range(int(os.environ.get("PLIES", "4"))):
    r = sp.roots.clone()
    sp.play_ply()
    ids, pi, k = (x.cpu().numpy() for x in sp.mcts.root_policy(r, None, 1.0))
    out[f"pi{i}"], out[f"ids{i}"], out[f"act{i}"] = pi, ids, sp.last_action.cpu().numpy()
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1])
