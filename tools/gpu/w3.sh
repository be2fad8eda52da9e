#!/bin/bash
# k_leafnet_w3: its parity tests, then the x3/w3 timing A/B. Later steps run only when pytest
# ended normally (0 passed / 1 failed): no GPU work after a fault, abort or time limit.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_leafnet_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_w3.log 2>&1
rc=$?; echo "leafnet pytest rc=$rc"; tail -25 gpurun_out/pytest_w3.log | cut -c1-300
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python tools/w3/bench_w3.py 100 3 > gpurun_out/bench_w3.json 2> gpurun_out/bench_w3.err
rc2=$?; echo "bench_w3 rc=$rc2"; cat gpurun_out/bench_w3.json; tail -5 gpurun_out/bench_w3.err
[ $rc2 -ne 0 ] && exit $rc2
if [ "$1" = "all" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_search_parity_gpu.py tests/test_vecenv_gpu.py tests/test_selfplay_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/newtests.log 2>&1
  rc3=$?; echo "newtests rc=$rc3"; tail -30 gpurun_out/newtests.log | cut -c1-300
  exit $rc3
fi
exit $rc
