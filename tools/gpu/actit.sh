#!/bin/bash
# the merged action table (one 16-B load per placement): bitwise tests, then self-play A/B vs the
# previous build (libbase.so), plies 5-30, and the fused-step stamps at ply 15
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/actit
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_mcts_gpu.py tests/test_sims_gpu.py tests/test_search_parity_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
BK_LIB=blokus_rl_amd/_lib/diag/libblokus_hip_diag.so timeout -k 10 200 python tools/stamp_step_ov.py 15 > $out/st15.json 2> $out/st.err || { tail $out/st.err; exit 1; }
STEPS=25 WARMUP=5 bash tools/gpu/lib_ab.sh "" blokus_rl_amd/_lib/exp/libprev.so blokus_rl_amd/_lib/exp/libbase.so
