#!/bin/bash
# Fused residual tower: conv GPU tests (incl. tower parity), tower timing, self-play bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_conv.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_conv.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/tower_bench.py 50 256 5 > gpurun_out/tower.json 2>gpurun_out/tower.err
rc=$?; echo "tower rc=$rc $(cat gpurun_out/tower.json)"
[ $rc -ne 0 ] && exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python bench.py --workload selfplay --no-cpu-baseline > gpurun_out/bench_sp.json 2> gpurun_out/bench_sp.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 gpurun_out/bench_sp.json
exit $rc
