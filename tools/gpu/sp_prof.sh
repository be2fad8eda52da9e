#!/bin/bash
# self-play bench alone (no CPU baselines), then the same under rocprofv3 --kernel-trace --stats
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload selfplay --no-cpu-baseline > gpurun_out/bench_sp.json 2> gpurun_out/bench_sp.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/bench_sp.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sp -o sp --output-format csv -- python bench.py --workload selfplay --no-cpu-baseline > gpurun_out/prof_sp.log 2>&1
rc=$?; echo "rocprof rc=$rc"; head -12 gpurun_out/prof_sp/sp_kernel_stats.csv | cut -c1-200
exit $rc
