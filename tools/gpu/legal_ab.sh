#!/bin/bash
# Legal-mask A/B of engine builds: tests/test_env_gpu.py per build (bit-exact against the oracle),
# then the classic kernel's time per launch at 4096 boards (tools/legal_scale.py) interleaved over
# ROUNDS rounds. Usage: bash tools/gpu/legal_ab.sh lib.so ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in "$@"; do
  BK_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_env_gpu.py \
    > gpurun_out/legal_ab_test.log 2>&1 || { echo "tests failed: $lib"; tail -20 gpurun_out/legal_ab_test.log; exit 1; }
  echo "tests ok: $lib $(tail -1 gpurun_out/legal_ab_test.log)"
done
for r in $(seq 1 ${ROUNDS:-3}); do
  for lib in "$@"; do
    out=$(BK_LIB=$lib timeout -k 10 120 python tools/legal_scale.py 4096) || exit 1
    echo "legal $lib $out"
  done
done
exit 0
