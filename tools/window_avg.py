"""Per-kernel average durations over the bench's timed self-play window from a rocprofv3 kernel
trace of `bench.py --steps S --warmup W`, next to the whole run's average. Every ply of the timed
run replays one graph with num_sims k_leaf_step_ov launches, so the window is that kernel's
dispatches [W*sims, (W+S)*sims) in trace order; the other kernels' window is the time span from the
end of the warmup's last leaf step to the end of the window's last one. Written for bench.py to read
(_window_trace) and committed under profiles/.
usage: python tools/window_avg.py <kernel_trace.csv> <out.json> <warmup> <steps> <sims> <games> <note>"""
import csv
import json
import sys

trace, out, note = sys.argv[1], sys.argv[2], sys.argv[7]
W, S, sims, games = (int(v) for v in sys.argv[3:7])
KERNELS = ("k_leaf_step_ov", "k_leafnet_x3", "k_select", "k_root", "k_ply")
seq = {k: [] for k in KERNELS}
with open(trace, newline="") as f:
    for r in csv.DictReader(f):
        name = r["Kernel_Name"]
        for k in KERNELS:
            if k in name:
                seq[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
                break
for v in seq.values():
    v.sort()
ls = seq["k_leaf_step_ov"]
t_lo = ls[W * sims - 1][1] if W > 0 else ls[0][0] - 1
t_hi = ls[(W + S) * sims - 1][1]
doc = {"round": 6, "note": note, "warmup": W, "steps": S, "sims": sims, "games": games,
       "window_span_ms": (t_hi - t_lo) / 1e6, "kernels": {}}
for k, v in seq.items():
    if not v:
        continue
    d = [(e - b) for b, e, _ in v]
    win = [(e - b) for b, e, _ in v if t_lo < b <= t_hi]
    doc["kernels"][k] = {"dispatches": len(d), "window_dispatches": len(win),
                         "window_avg_us": sum(win) / len(win) / 1e3 if win else None,
                         "window_total_ms": sum(win) / 1e6, "run_avg_us": sum(d) / len(d) / 1e3,
                         "names": sorted({n[:80] for _, _, n in v})[:4]}
assert doc["kernels"]["k_leaf_step_ov"]["window_dispatches"] == S * sims, doc["kernels"]["k_leaf_step_ov"]
json.dump(doc, open(out, "w"), indent=1)
print(json.dumps({k: {a: b for a, b in v.items() if a != "names"} for k, v in doc["kernels"].items()}))
