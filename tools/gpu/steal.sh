#!/bin/bash
# k_leaf_step_ws (logits shared across workgroups) vs k_leaf_step_ov: bitwise tests, then self-play
# sims/s interleaved (plies 5-30)
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/steal
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_sims_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
grep -E "passed|failed" $out/pytest.log | tail -2
BK_STEP_STEAL=1 timeout -k 10 300 python -u -m pytest tests/test_search_parity_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/pytest2.log 2>&1 || { tail -30 $out/pytest2.log; exit 1; }
tail -1 $out/pytest2.log
for i in 1 2; do
  for s in 0 1; do
    BK_STEP_STEAL=$s timeout -k 10 300 python bench.py --workload selfplay --no-cpu-baseline > $out/sp_${s}_$i.json 2> $out/sp.err || { tail $out/sp.err; exit 1; }
    python -c "import json; d=json.load(open('$out/sp_${s}_$i.json')); print('steal $s', round(d['value']), round(d['ms_per_step'],3), 'ms/ply; leaf step', round(d['search_roofline']['k_leaf_step_us'],1), 'us')"
  done
done
