"""Diagnostic: k_legal_mask time per launch vs batch size (graph of back-to-back launches, HIP
events), to tell per-wave latency from throughput limits. Run under rocprofv3 --kernel-trace --stats
for the kernels' own durations."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from blokus_rl_amd.boards import random_boards  # noqa: E402
from blokus_rl_amd.engine import Engine  # noqa: E402

eng = Engine(20, 4, 5)
out = {}
for B in [int(x) for x in (sys.argv[1:] or ["1024", "2048", "4096", "8192", "16384"])]:
    states = random_boards(eng, B, seed0=0)
    masks = torch.empty((B, eng.W), dtype=torch.int64, device=eng.device)
    counts = torch.empty(B, dtype=torch.int32, device=eng.device)
    st = torch.cuda.current_stream()
    s = torch.cuda.Stream()
    s.wait_stream(st)
    with torch.cuda.stream(s):
        eng.legal_mask_into(states, masks, counts)
    st.wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            eng.legal_mask_into(states, masks, counts)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(10):
        g.replay()
    e1.record(st)
    torch.cuda.synchronize()
    out[B] = round(e0.elapsed_time(e1) * 1e3 / 200, 2)
print(json.dumps({"us_per_launch": out}))
