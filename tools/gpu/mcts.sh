#!/bin/bash
# GPU step: MCTS + env parity tests, then a rocprofv3 kernel-trace of the legal-move bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_legal -o legal --output-format csv -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --graph 0 > gpurun_out/prof_legal.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_legal.log
find gpurun_out/prof_legal -name "*stats*" | head
exit $rc
