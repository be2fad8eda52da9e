#!/bin/bash
# Round validation on one MI355X: GPU tests, smoke(), the default bench, and the bench under
# rocprofv3 --kernel-trace --stats (the committed kernel summary). Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_all.json 2> gpurun_out/bench_all.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 gpurun_out/bench_all.json
[ $rc -ne 0 ] && exit $rc
[ -n "$NO_PROF" ] && exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_all -o all --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof_all.log 2>&1
rc=$?; echo "rocprof rc=$rc"; head -20 gpurun_out/prof_all/all_kernel_stats.csv | cut -c1-160
exit $rc
