#!/bin/bash
# Full default bench (as the driver runs it) + selfplay GPU tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_selfplay_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_sp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_sp.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_all.json 2> gpurun_out/bench_all.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_all.json; grep -v amdgpu.ids gpurun_out/bench_all.err | tail -5
exit $rc
