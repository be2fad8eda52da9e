#!/bin/bash
# Search, self-play and conv GPU tests (the fused leaf step and graph replay), the self-play bench line, and
# its kernel-trace summary.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_sims_gpu.py tests/test_selfplay_gpu.py tests/test_mcts_gpu.py tests/test_conv_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sims.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_sims.log | cut -c1-150 | tail -30; tail -3 gpurun_out/pytest_sims.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload selfplay --no-cpu-baseline > gpurun_out/bench_sims.json 2> gpurun_out/bench_sims.err
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.load(open('gpurun_out/bench_sims.json')); r=d['roofline']; print(d['value'], r.get('kernel_ms'), r.get('achieved'), r.get('frac'), r.get('share_of_ply')); print(d['stage_ms_per_sim_step'])"
[ $rc -ne 0 ] && exit $rc
[ -n "$NO_PROF" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sims -o sp --output-format csv -- python bench.py --workload selfplay --no-cpu-baseline > gpurun_out/prof_sims.log 2>&1
rc=$?; echo "rocprof rc=$rc"
python - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/prof_sims/sp_kernel_stats.csv')))[:10]:
    print(r['Name'].replace('(anonymous namespace)::', '').split('(')[0][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
exit $rc
