#!/bin/bash
# The learner workload (§8f row 1) under rocprofv3 --kernel-trace --stats: where a train step's
# time goes (MIOpen convolutions, BN, GEMMs, loss kernels, Adam).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload train --no-cpu-baseline > gpurun_out/learner.json 2> gpurun_out/learner.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/learner.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_learner -o learner --output-format csv -- python bench.py --workload train --no-cpu-baseline > gpurun_out/prof_learner.log 2>&1
rc=$?; echo "rocprof rc=$rc"; head -25 gpurun_out/prof_learner/learner_kernel_stats.csv | cut -c1-200
exit $rc
