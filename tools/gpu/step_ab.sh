#!/bin/bash
# GPU session: new/changed tests, the wx3 A/B timing, and self-play with and without the
# overlapped leaf step. Stops at the first step that ends in anything but pass/fail (fault,
# abort, timeout).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
TESTS=${TESTS:-"tests/test_sims_gpu.py tests/test_search_parity_gpu.py tests/test_dropin_gpu.py tests/test_selfplay_gpu.py"} bash tools/gpu/newtests.sh
rc=$?; ok $rc || exit $rc
timeout -k 10 120 python tools/wx3_bench.py > gpurun_out/wxb.log 2>&1
rc=$?; tail -3 gpurun_out/wxb.log; ok $rc || exit $rc
timeout -k 10 200 python bench.py --workload selfplay --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/sp_ov.json 2> gpurun_out/sp_ov.err
rc=$?; cut -c1-300 gpurun_out/sp_ov.json; [ $rc -eq 0 ] || exit $rc
BK_STEP_OVERLAP=0 timeout -k 10 200 python bench.py --workload selfplay --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/sp_noov.json 2> gpurun_out/sp_noov.err
rc=$?; cut -c1-300 gpurun_out/sp_noov.json; exit $rc
