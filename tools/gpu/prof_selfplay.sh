#!/bin/bash
# kernel-trace stats of a short self-play bench (env passes through, e.g. BK_LEAF_AM=0);
# prints the engine kernels' average durations. Usage: prof_selfplay.sh <name>
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
n=${1:-sp}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$n -o $n --output-format csv -- python bench.py --workload selfplay --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/prof_$n.log 2>&1 || { tail -5 gpurun_out/prof_$n.log; exit 1; }
python - "$n" <<'PY'
import csv, sys
n = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/prof_{n}/{n}_kernel_stats.csv")):
    name = r["Name"]
    if "bk::" in name:
        print(n, name.split("(")[0][-40:], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1))
PY
