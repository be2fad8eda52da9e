#!/bin/bash
# leaf logits through the all-loads-first register path (libreg: -DBK_LEAF_REG=1): the leaf-step
# parity tests under it, then driver-argument self-play (20 plies after 5), interleaved with the
# in-tree build
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/reg
BK_LIB=blokus_rl_amd/_lib/exp/libreg.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sims_gpu.py tests/test_search_parity_gpu.py > gpurun_out/reg/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/reg/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in "" blokus_rl_amd/_lib/exp/libreg.so; do
    BK_LIB=$lib timeout -k 10 300 python bench.py --workload selfplay --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/reg/b.json 2> gpurun_out/reg/b.err || { tail -5 gpurun_out/reg/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/reg/b.json')); print('lib [%s]' % sys.argv[1], round(d['value']), round(d['ms_per_step'],3))" "$lib"
  done
done
