#!/bin/bash
# search-kernel change check: the MCTS/self-play/drop-in GPU tests, then the self-play bench and
# the per-phase stamps of k_select / k_expand_backup (diagnostic build)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mcts_gpu.py tests/test_sims_gpu.py tests/test_selfplay_gpu.py tests/test_dropin_gpu.py tests/test_arena_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_search.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_search.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/pytest_search.log | head -20; exit $rc; }
tools/gpu/sp_variants.sh || exit 1
BK_LIB=blokus_rl_amd/_lib/diag/libblokus_hip_diag.so timeout -k 10 300 python tools/stamp_search.py
