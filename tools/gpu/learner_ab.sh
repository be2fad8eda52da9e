#!/bin/bash
# Learner A/B of engine builds: the bench's learner line (batch 1024) per library, interleaved
# (ROUNDS rounds; "" = the in-tree default). Usage: bash tools/gpu/learner_ab.sh "" lib.so ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    BK_LIB=$lib timeout -k 10 300 python bench.py --workload train --steps 20 --warmup 5 --no-cpu-baseline \
      > gpurun_out/lab.json 2> gpurun_out/lab.err || { echo "failed: $lib"; tail -5 gpurun_out/lab.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/lab.json')); d=d.get('learner', d); print('lib [%s]' % sys.argv[1], round(d['value']), 'ms', round(d['ms_per_step'],3))" "$lib"
  done
done
