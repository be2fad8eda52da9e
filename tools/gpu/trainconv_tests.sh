#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_train_conv_gpu.py tests/test_learner.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tc_only.log 2>&1
rc=$?; tail -3 gpurun_out/tc_only.log; exit $rc
