#!/bin/bash
# Round validation: every GPU test, smoke(), the default bench, then the same bench under
# rocprofv3 --kernel-trace --stats. Outputs under gpurun_out/; copy the summaries to profiles/.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_all.json 2> gpurun_out/bench_all.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 gpurun_out/bench_all.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_all -o all --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof_all.log 2>&1
rc=$?; echo "rocprof rc=$rc"; head -14 gpurun_out/prof_all/all_kernel_stats.csv | cut -c1-160
exit $rc
