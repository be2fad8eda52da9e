#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_selfplay_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_sp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_sp.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --workload selfplay --steps 3 --warmup 1 > gpurun_out/bench_sp.json 2> gpurun_out/bench_sp.err
rc=$?; echo "bench resnet rc=$rc"; cat gpurun_out/bench_sp.json; tail -5 gpurun_out/bench_sp.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --workload selfplay --model dumbnet --steps 3 --warmup 1 > gpurun_out/bench_sp_dumb.json 2> gpurun_out/bench_sp_dumb.err
rc=$?; echo "bench dumbnet rc=$rc"; cat gpurun_out/bench_sp_dumb.json; tail -5 gpurun_out/bench_sp_dumb.err
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sp -o sp --output-format csv -- python bench.py --workload selfplay --steps 2 --warmup 1 > gpurun_out/prof_sp.log 2>&1
rc=$?; echo "rocprof rc=$rc"; head -25 gpurun_out/prof_sp/sp_kernel_stats.csv | cut -c1-200
exit $rc
