#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sims_gpu.py tests/test_mcts_gpu.py tests/test_selfplay_gpu.py tests/test_dropin_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_step.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_step.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_step.log | head -20; exit $rc; }
SP_STEPS=10 tools/gpu/sp_variants.sh
