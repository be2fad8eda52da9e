#!/bin/bash
# x3 leaf-net kernel: its parity tests, then every GPU test, then the default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_leafnet_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_leafnet.log 2>&1
rc=$?; echo "leafnet pytest rc=$rc"; tail -15 gpurun_out/pytest_leafnet.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_all.json 2> gpurun_out/bench_all.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench_all.json
exit $rc
