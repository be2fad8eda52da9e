#!/bin/bash
# legal-mask change check: env/MCTS GPU tests, the config-2 legal-move bench, self-play bench, search stamps
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_mcts_gpu.py tests/test_sims_gpu.py tests/test_selfplay_gpu.py tests/test_dropin_gpu.py tests/test_vecenv_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_legal.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_legal.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/pytest_legal.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --workload legal --no-cpu-baseline > gpurun_out/bench_legal.json 2> gpurun_out/bench_legal.err || { tail gpurun_out/bench_legal.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_legal.json')); print('legal', round(d['value']/1e6,1), 'M boards/s', d['roofline'])"
tools/gpu/sp_variants.sh || exit 1
BK_LIB=blokus_rl_amd/_lib/diag/libblokus_hip_diag.so timeout -k 10 300 python tools/stamp_search.py
