#!/bin/bash
# W-row loads skipped where the policy features are zero (BK_LEAF_SKIP0=1): bitwise tests against the
# stagewise path and the oracle replays, then self-play sims/s interleaved (plies 5-30) and the ply-15 stamps
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/skip0
mkdir -p $out
BK_LEAF_SKIP0=1 timeout -k 10 400 python -u -m pytest tests/test_sims_gpu.py tests/test_search_parity_gpu.py tests/test_selfplay_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
BK_LEAF_SKIP0=1 BK_LIB=blokus_rl_amd/_lib/diag/libblokus_hip_diag.so timeout -k 10 200 python tools/stamp_step_ov.py 15 > $out/st15.json 2> $out/st.err || { tail $out/st.err; exit 1; }
for i in 1 2; do
  for s in 0 1; do
    BK_LEAF_SKIP0=$s timeout -k 10 300 python bench.py --workload selfplay --no-cpu-baseline --late-plies 0 > $out/sp_${s}_$i.json 2> $out/sp.err || { tail $out/sp.err; exit 1; }
    python -c "import json; d=json.load(open('$out/sp_${s}_$i.json')); print('skip0 $s', round(d['value']), round(d['ms_per_step'],3), 'ms/ply; leaf step', round(d['search_roofline']['k_leaf_step_us'],1), 'us')"
  done
done
