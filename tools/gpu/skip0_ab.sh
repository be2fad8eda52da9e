#!/bin/bash
# A/B: LDS atomics only for non-zero fields (default) vs every lane (libskip0off.so): bit-exact
# tests, then the legal-move and self-play benches with both libraries.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s0
TESTS="tests/test_env_gpu.py tests/test_sims_gpu.py tests/test_search_parity_gpu.py" bash tools/gpu/newtests.sh
rc=$?; [ $rc -eq 0 ] || exit $rc
for lib in "" blokus_rl_amd/_lib/exp/libskip0off.so; do
  BK_LIB=$lib timeout -k 10 120 python bench.py --workload legal --no-cpu-baseline > gpurun_out/s0/l.json 2> gpurun_out/s0/l.err || { tail -3 gpurun_out/s0/l.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s0/l.json')); r=d['roofline']; print('legal lib [$lib]', round(r['kernel_ms']*1e3,2), 'us', round(r['frac'],3))"
  BK_LIB=$lib timeout -k 10 200 python bench.py --workload selfplay --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/s0/s.json 2> gpurun_out/s0/s.err || { tail -3 gpurun_out/s0/s.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s0/s.json')); print('selfplay lib [$lib]', round(d['value']), 'step_us', round(d['search_roofline']['k_leaf_step_us'],1))"
done
