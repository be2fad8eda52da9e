"""Summarise a rocprofv3 kernel_stats.csv per step: python tools/prof_summary.py <csv> <steps> [top]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
tot = 0.0
for r in rows[:top]:
    us = int(r["TotalDurationNs"]) / steps / 1000
    tot += us
    print(f"{r['Name'][:80]:80s} calls/step={int(r['Calls']) / steps:6.2f} us/step={us:8.1f} "
          f"avg={float(r['AverageNs']) / 1000:7.1f}")
print("total (top rows) us/step", round(tot, 1))
