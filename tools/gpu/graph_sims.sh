#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/spvar; mkdir -p $out
for k in 10 25 50 100; do
  BK_SIM_GRAPH_SIMS=$k timeout -k 10 300 python bench.py --workload selfplay --no-cpu-baseline --steps 10 --warmup 2 > $out/g$k.json 2> $out/g$k.err || { echo "$k failed"; tail -5 $out/g$k.err; exit 1; }
  python -c "import json; d=json.load(open('$out/g$k.json')); print('graph sims $k', round(d['value']))"
done
