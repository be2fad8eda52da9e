#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_search_parity_gpu.py tests/test_vecenv_gpu.py tests/test_selfplay_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/newtests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/newtests.log
exit $rc
