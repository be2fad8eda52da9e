"""Fold rocprofv3 --pmc pass directories into a profiles/*pmc*.json entry that bench.py reads
(_pmc_traffic): per-dispatch means of every counter for kernels whose name contains <pattern>,
HBM bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (the gfx950 FETCH_SIZE correction of
MI355X_MICROARCH.md §HBM; both counters are in KB). <pattern> is a regular expression searched in
the kernel name. BK_PMC_RANGE=lo:hi keeps only the matching dispatches lo..hi-1 in dispatch order
(e.g. the bench's timed window of plies); BK_PMC_SCALE multiplies the bytes (a launch pair: 2).
usage: python tools/pmc_to_json.py <out.json> <key> <pattern> <units_per_launch> <algorithmic_bytes> <note> <pass dirs...>"""
import collections
import csv
import glob
import json
import os
import re
import sys

out, key, pat, units, algo, note = sys.argv[1:7]
dirs = sys.argv[7:]
acc = collections.defaultdict(list)
rx = re.compile(pat)
rng = os.environ.get("BK_PMC_RANGE")
lo, hi = (int(v) for v in rng.split(":")) if rng else (0, 1 << 62)
for d in dirs:
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if rx.search(r.get("Kernel_Name", ""))]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    keep = set(ids[lo:hi])
    for r in rows:
        if int(r["Dispatch_Id"]) in keep:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
means = {k: sum(v) / len(v) for k, v in acc.items()}
scale = float(os.environ.get("BK_PMC_SCALE", "1"))  # e.g. 2: a launch pair of two kernels
fetch = 2 * means.get("FETCH_SIZE", 0.0) * 1024 * scale
write = means.get("WRITE_SIZE", 0.0) * 1024 * scale
rnd = int(os.environ.get("BK_PMC_ROUND", "6"))
doc = json.load(open(out)) if os.path.exists(out) else {"round": rnd, "kernels": {}}
doc["round"] = max(int(doc.get("round", rnd)), rnd)
doc.setdefault("notes", {})[key] = note
doc["kernels"][key] = {"units_per_launch": int(units), "hbm_bytes_per_launch": fetch + write, "fetch_bytes": fetch,
                       "write_bytes": write, "algorithmic_bytes": int(float(algo)), "dispatches": len(acc.get("FETCH_SIZE", [])),
                       "kernel_pattern": pat, "dispatch_range": rng, "counters_per_dispatch": means}
json.dump(doc, open(out, "w"), indent=1)
print(key, {k: (round(v, 1) if isinstance(v, float) else v) for k, v in doc["kernels"][key].items()
           if k != "counters_per_dispatch"})
