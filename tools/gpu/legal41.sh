#!/bin/bash
# config-2 piece-list legal kernel (BK_LEGAL_WPB=41): bit-exact vs the oracle, then timed beside the default
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/legal41
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_env_gpu.py -k "variants" > gpurun_out/legal41/test.log 2>&1 || { tail -30 gpurun_out/legal41/test.log; exit 1; }
tail -3 gpurun_out/legal41/test.log
BK_LEGAL_VARIANTS="1 41 42 43 1 41" bash tools/gpu/legal_variants.sh
