"""Launch gaps of the self-play sim-step from a rocprofv3 kernel trace (tools/gpu/gaps_selfplay.sh):
median idle time between the end of one engine kernel and the start of the next, per kernel pair,
and the share of the timed window the GPU spends between kernels.
Usage: python tools/trace_gaps.py <kernel_trace.csv>"""
import collections
import csv
import json
import sys

import numpy as np


def short(name: str) -> str:
    for k in ("k_leafnet_x3", "k_leaf_step", "k_select", "k_root", "k_next_state", "k_game_ended",
              "k_expand_backup", "k_leaf_logits"):
        if k in name:
            return k
    return "other"


rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
# the timed plies: the last stretch of leaf-net launches (skip warm-up / model build)
ln = [i for i, e in enumerate(ev) if e[2] == "k_leafnet_x3"]
lo = ln[len(ln) // 4]
win = ev[lo:ln[-1] + 2]
gaps = collections.defaultdict(list)
busy = 0
for a, b in zip(win, win[1:]):
    gaps[(a[2], b[2])].append((b[0] - a[1]) / 1e3)
for s, e, _ in win:
    busy += e - s
span = win[-1][1] - win[0][0]
out = {"window_us": span / 1e3, "kernel_busy_frac": busy / span,
       "gap_us_median": {f"{k[0]}->{k[1]}": [round(float(np.median(v)), 2), len(v)] for k, v in gaps.items() if len(v) >= 3}}
print(json.dumps(out, indent=1))
# where the window's time goes: per kernel class (busy us) and the idle time between kernels
cls = collections.defaultdict(float)
cnt = collections.Counter()
for s, e, k in win:
    cls[k] += (e - s) / 1e3
    cnt[k] += 1
idle = sum((b[0] - a[1]) / 1e3 for a, b in zip(win, win[1:]) if b[0] > a[1])
plies = max(1, cnt["k_root"])
print(json.dumps({"plies_in_window": plies, "busy_us_per_ply": {k: round(v / plies, 1) for k, v in cls.items()},
                  "launches_per_ply": {k: round(v / plies, 1) for k, v in cnt.items()},
                  "idle_us_per_ply": round(idle / plies, 1)}, indent=1))
