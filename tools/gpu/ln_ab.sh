#!/bin/bash
# Leaf-net A/B of engine builds: the leaf-net GPU tests per build, then k_leafnet_x3's time per
# launch (tools/leafnet_bench.py, 256 boards) interleaved (ROUNDS rounds), then the self-play A/B
# (tools/gpu/lib_ab.sh). Usage: bash tools/gpu/ln_ab.sh lib.so ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in "$@"; do
  BK_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_leafnet_gpu.py \
    > gpurun_out/ln_ab_test.log 2>&1 || { echo "tests failed: $lib"; tail -20 gpurun_out/ln_ab_test.log; exit 1; }
  echo "tests ok: $lib $(tail -1 gpurun_out/ln_ab_test.log)"
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    BK_LIB=$lib timeout -k 10 120 python tools/leafnet_bench.py 300 256 > gpurun_out/lnb.json || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/lnb.json')); print('leafnet', sys.argv[1], round(d['us_per_launch'],2))" "$lib"
  done
done
[ "${SELFPLAY:-1}" = "1" ] && bash tools/gpu/lib_ab.sh "$@"
exit 0
