#!/bin/bash
# Round 6, §8f row 4: PPO GPU tests, the PPO bench leg (MIOPEN_FIND_MODE=FAST) and the
# kernel-trace stats of one update (-> gpurun_out/r06_ppo_kernel_stats.csv).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ppo.py > gpurun_out/r06_ppo_tests.log 2>&1 \
  || { tail -30 gpurun_out/r06_ppo_tests.log; exit 1; }
tail -2 gpurun_out/r06_ppo_tests.log
export MIOPEN_FIND_MODE=FAST
timeout -k 10 400 python bench.py --workload ppo > gpurun_out/r06_ppo_bench.json 2> gpurun_out/r06_ppo_bench.err \
  || { tail -20 gpurun_out/r06_ppo_bench.err; exit 1; }
cat gpurun_out/r06_ppo_bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/r06_ppo_prof -o ppo --output-format csv -- python bench.py --workload ppo --ppo-updates 1 --no-cpu-baseline > gpurun_out/r06_ppo_prof.log 2>&1 || { tail -5 gpurun_out/r06_ppo_prof.log; exit 1; }
find /tmp/r06_ppo_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r06_ppo_kernel_stats.csv \;
head -8 gpurun_out/r06_ppo_kernel_stats.csv | cut -c1-150
