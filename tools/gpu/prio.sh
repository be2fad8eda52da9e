#!/bin/bash
# wave 0 of k_leaf_step_ov at issue priority 3 (BK_STEP_PRIO=1) vs 0: bitwise tests, stamps at ply 15,
# self-play sims/s interleaved (plies 5-30)
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/prio
mkdir -p $out
BK_STEP_PRIO=1 timeout -k 10 300 python -u -m pytest tests/test_sims_gpu.py tests/test_search_parity_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
BK_STEP_PRIO=1 BK_LIB=blokus_rl_amd/_lib/diag/libblokus_hip_diag.so timeout -k 10 200 python tools/stamp_step_ov.py 15 > $out/st15.json 2> $out/st.err || { tail $out/st.err; exit 1; }
for i in 1 2; do
  for s in 0 1; do
    BK_STEP_PRIO=$s timeout -k 10 300 python bench.py --workload selfplay --no-cpu-baseline --late-plies 0 > $out/sp_${s}_$i.json 2> $out/sp.err || { tail $out/sp.err; exit 1; }
    python -c "import json; d=json.load(open('$out/sp_${s}_$i.json')); print('prio $s', round(d['value']), round(d['ms_per_step'],3), 'ms/ply; leaf step', round(d['search_roofline']['k_leaf_step_us'],1), 'us')"
  done
done
