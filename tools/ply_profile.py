"""Per-ply breakdown of a self-play kernel trace (tools/gpu/ply_profile.sh): for each ply (one
captured graph: k_select, then 100 x {k_leafnet_x3, k_leaf_step}), the span, the leaf-net and
leaf-step time, and the tail (everything between the last leaf step and the next k_select).
Usage: python tools/ply_profile.py <kernel_trace.csv>"""
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
sel = [i for i, e in enumerate(ev) if "k_select(" in e[2]]
out = []
for a, b in zip(sel, sel[1:]):
    seg = ev[a:b]
    nets = [(e[1] - e[0]) / 1e3 for e in seg if "k_leafnet_x3" in e[2]]
    steps = [(e[1] - e[0]) / 1e3 for e in seg if "k_leaf_step" in e[2]]
    if len(nets) < 90:
        continue
    last = max(i for i, e in enumerate(seg) if "k_leaf_step" in e[2])
    tail = (ev[b][0] - seg[last][1]) / 1e3
    out.append({"span_ms": round((ev[b][0] - ev[a][0]) / 1e6, 3), "net_us": round(sum(nets) / len(nets), 1),
                "step_us": round(sum(steps) / len(steps), 1), "step_max_us": round(max(steps), 1),
                "tail_us": round(tail, 1)})
print(json.dumps(out, indent=0))
