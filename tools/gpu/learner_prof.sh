#!/bin/bash
# Kernel-trace stats of the learner's device path alone (tools/learner_pmc.py: batch 1024, 13
# train steps + the conv kernels' timing loops) -> gpurun_out/learner_kernel_stats.csv.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ln_kt -o ln --output-format csv -- python tools/learner_pmc.py ${1:-10} \
  > gpurun_out/learner_prof.log 2>&1 || { tail -5 gpurun_out/learner_prof.log; exit 1; }
find /tmp/ln_kt -name "*kernel_stats.csv" -exec cp {} gpurun_out/learner_kernel_stats.csv \;
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/learner_kernel_stats.csv")))
for r in rows[:45]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:100]}")
PY
