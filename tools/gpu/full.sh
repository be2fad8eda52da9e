#!/bin/bash
# Full default bench + rocprof kernel-trace of the default bench (the committed profile).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_all.json 2> gpurun_out/bench_all.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_all.json; grep -v amdgpu.ids gpurun_out/bench_all.err | tail -3
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_all -o all --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof_all.log 2>&1
rc=$?; echo "rocprof rc=$rc"; head -30 gpurun_out/prof_all/all_kernel_stats.csv | cut -c1-180
exit $rc
