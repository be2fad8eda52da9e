#!/bin/bash
# Round 6, config 5: the masked-policy draw (bk_vec_policy) — GPU tests, the vecenv bench line,
# PMC passes of k_vec_step7 (headline mode) and k_vec_policy (each to its own summary file).
#   tools/gpu/r06_vec.sh [pytest -k expression]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
K=${1:-"vec or policy or ppo or capi"}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_vecenv_gpu.py tests/test_capi.py \
  tests/test_ppo.py -k "$K" > gpurun_out/r06_vec_tests.log 2>&1 || { tail -30 gpurun_out/r06_vec_tests.log; exit 1; }
tail -3 gpurun_out/r06_vec_tests.log
timeout -k 10 300 python bench.py --workload vecenv --no-cpu-baseline > gpurun_out/r06_vec_bench.json 2> gpurun_out/r06_vec_bench.err \
  || { tail -20 gpurun_out/r06_vec_bench.err; exit 1; }
cat gpurun_out/r06_vec_bench.json
tools/gpu/pmc_kernel.sh gpurun_out/r06_pmc_vec_step7.json k_vec_step7 k_vec_step7 8192 3219456 \
  "round 6: rocprofv3 --pmc passes of tools/vec_pmc.py random (eager k_vec_step7, in-kernel agent draws, 8192 envs, 70 launches); algorithmic bytes = 8192 x 393" \
  120 -- python tools/vec_pmc.py random 50 || exit 1
tools/gpu/pmc_kernel.sh gpurun_out/r06_pmc_vec_policy.json k_vec_step7_policy "k_vec_step7<4, 16, 2>|k_vec_step7ILi4ELi16ELi2E" 8192 0 \
  "round 6: rocprofv3 --pmc passes of tools/vec_pmc.py policy (eager fused draw + step, k_vec_step7<4,16,2>, 8192 envs, 70 launches); algorithmic bytes per env: 393 + 4 x the legal ids + 8 (the bench line's bytes_per_unit)" \
  120 -- python tools/vec_pmc.py policy 50 || exit 1
tools/gpu/pmc_kernel.sh gpurun_out/r06_pmc_vec_draw.json k_vec_policy k_vec_policy 8192 0 \
  "round 6: rocprofv3 --pmc passes of tools/vec_pmc.py draw (eager standalone k_vec_policy, 16 lanes per env, 8192 envs, 70 launches); algorithmic bytes per env: 4 x the legal ids + 120 mask + 16 rng + 8 out (the bench line's draw_alone.bytes_per_unit)" \
  120 -- python tools/vec_pmc.py draw 50 || exit 1
echo ALLOK
