#!/bin/bash
# GPU tests in one process, each under the per-test time limit, stopping at the first failure.
#   tools/gpu/tests.sh [pytest args...]      (default: the whole -m gpu suite)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "${@:-tests}" \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/gpu_tests.log | grep -c PASSED
tail -5 gpurun_out/gpu_tests.log
exit $rc
