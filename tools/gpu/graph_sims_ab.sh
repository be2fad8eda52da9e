#!/bin/bash
# A/B of the simulations per captured graph (BK_SIM_GRAPH_SIMS; 0 = the default: the whole ply)
cd "$GRAFT_REPO_ROOT" || exit 1
for k in ${GRAPH_SIMS_LIST:-10 100 10 100}; do
  BK_SIM_GRAPH_SIMS=$k timeout -k 10 200 python bench.py --workload selfplay --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/ab_$k.json 2> gpurun_out/ab_$k.err || { tail -3 gpurun_out/ab_$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$k.json')); print('graph sims $k', round(d['value']))"
done
