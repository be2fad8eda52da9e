#!/bin/bash
# instruction-cache counters of the self-play kernels (one --pmc pass; the short self-play bench)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_ic
timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES --output-format csv -d gpurun_out/pmc_ic -o ic -- python bench.py --workload selfplay --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/pmc_ic.log 2>&1 || { tail -5 gpurun_out/pmc_ic.log; exit 1; }
python - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_ic/**/*counter_collection.csv", recursive=True)
print(f)
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for path in f:
    for r in csv.DictReader(open(path)):
        k = r.get("Kernel_Name", r.get("Kernel-Name", ""))
        if "bk::" not in k and "leafnet" not in k:
            continue
        name = k.split("(")[0][-30:]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(name, r["Counter_Name"])] += 1
for name, d in agg.items():
    n = max(cnt[(name, c)] for c in d)
    print(name, "launches", n, {c: round(v / n) for c, v in d.items()})
PY
