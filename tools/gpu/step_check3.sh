#!/bin/bash
# GPU session: the search tests, the leaf-step stamps (diag build) and an interleaved self-play A/B
# of the libraries given as arguments ("" = the default build).
cd "$GRAFT_REPO_ROOT" || exit 1
TESTS="tests/test_sims_gpu.py tests/test_search_parity_gpu.py tests/test_mcts_gpu.py tests/test_selfplay_gpu.py" bash tools/gpu/newtests.sh || exit 1
BK_LIB=blokus_rl_amd/_lib/diag/libblokus_hip_diag.so timeout -k 10 200 python tools/stamp_step_ov.py 6 > gpurun_out/stov.log 2>&1 || exit 1
tail -1 gpurun_out/stov.log | cut -c1-700
bash tools/gpu/lib_ab.sh "$@"
