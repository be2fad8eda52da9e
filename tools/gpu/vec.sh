#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_vecenv_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_vec.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_vec.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --workload vecenv > gpurun_out/bench_vec.json 2> gpurun_out/bench_vec.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_vec.json; grep -v amdgpu.ids gpurun_out/bench_vec.err | tail -3
exit $rc
