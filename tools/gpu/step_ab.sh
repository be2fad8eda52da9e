#!/bin/bash
# leaf-step change: the search parity tests on the in-tree build, then self-play sims/s of the
# in-tree build vs blokus_rl_amd/_lib/exp/libprev.so (tools/gpu/lib_ab.sh, 3 rounds)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/step
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sims_gpu.py tests/test_search_parity_gpu.py tests/test_mcts_gpu.py > gpurun_out/step/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/step/pytest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash tools/gpu/lib_ab.sh "" blokus_rl_amd/_lib/exp/libprev.so
