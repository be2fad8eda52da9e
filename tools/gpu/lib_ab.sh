#!/bin/bash
# Self-play sims/s of several engine builds, interleaved (ROUNDS rounds; BK_LIB per run; "" = the
# default in-tree library; STEPS / WARMUP plies, default 6 / 2). Usage: bash tools/gpu/lib_ab.sh "" blokus_rl_amd/_lib/exp/libX.so ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    BK_LIB=$lib timeout -k 10 200 python bench.py --workload selfplay --steps ${STEPS:-6} --warmup ${WARMUP:-2} --late-plies 0 --no-cpu-baseline \
      > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "failed: $lib"; tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('lib [%s]' % sys.argv[1], round(d['value']), 'step_us', round(d['search_roofline']['k_leaf_step_us'],1))" "$lib"
  done
done
