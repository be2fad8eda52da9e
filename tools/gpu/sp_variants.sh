#!/bin/bash
# self-play bench (5 timed plies) with the in-tree library and each blokus_rl_amd/_lib/exp/libln_*.so
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/spvar; mkdir -p $out
run() {
  timeout -k 10 300 python bench.py --workload selfplay --no-cpu-baseline --steps ${SP_STEPS:-5} --warmup 2 > $out/$1.json 2> $out/$1.err || { echo "$1 failed"; tail -5 $out/$1.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$out/$1.json')); print('$1', round(d['value']), {k: round(v*1e3,1) for k,v in d['stage_ms_per_sim_step'].items()}, 'kernel_us', round(d['roofline']['kernel_ms']*1e3,1))"
}
run intree
for lib in $(ls blokus_rl_amd/_lib/exp/libln_*.so 2>/dev/null); do
  n=$(basename $lib .so)
  BK_LIB=$lib run $n
done
