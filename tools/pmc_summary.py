"""Mean PMC counter values (and kernel durations) per kernel-name filter from rocprofv3 CSVs:
python tools/pmc_summary.py <dir-with-p*/> <kernel-substring>."""
import collections
import csv
import glob
import sys

d, pat = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{d}/p*/*counter_collection.csv")):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if pat in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/")[-2], {k: round(sum(v) / len(v), 1) for k, v in acc.items()})
for f in sorted(glob.glob(f"{d}/p*/*kernel_trace.csv"))[:1]:
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(f))
            if pat in r.get("Kernel_Name", "")]
    print("kernel ns (profiled run) mean", sum(durs) / len(durs), "n", len(durs))
