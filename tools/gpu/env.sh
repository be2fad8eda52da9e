#!/bin/bash
# GPU step: parity tests, then the legal-move bench. Stops at the first fault-like exit.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 5 > gpurun_out/bench_legal.json 2> gpurun_out/bench_legal.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_legal.json; tail -5 gpurun_out/bench_legal.err
exit $rc
