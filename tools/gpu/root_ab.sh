#!/bin/bash
# k_root change: the root-policy / MCTS parity tests, then 12-ply self-play runs (late plies have
# the long root rows) of the in-tree build vs blokus_rl_amd/_lib/exp/libprev.so, interleaved
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/root
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mcts_gpu.py tests/test_dropin_gpu.py tests/test_selfplay_gpu.py tests/test_arena_gpu.py > gpurun_out/root/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/root/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in "" blokus_rl_amd/_lib/exp/libprev.so; do
    BK_LIB=$lib timeout -k 10 300 python bench.py --workload selfplay --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/root/b.json 2> gpurun_out/root/b.err || { tail -5 gpurun_out/root/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/root/b.json')); print('lib [%s]' % sys.argv[1], round(d['value']), round(d['ms_per_step'],3))" "$lib"
  done
done
