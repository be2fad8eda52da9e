#!/bin/bash
# Quick GPU run of a list of test files (default: the tests touched this session).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TESTS:-"tests/test_mcts_gpu.py tests/test_leafnet_gpu.py tests/test_dist_gpu.py tests/test_dropin_gpu.py tests/test_selfplay_gpu.py"}
timeout -k 10 500 python -u -m pytest $T -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_new.log | tail -40
exit $rc
