#!/bin/bash
# Self-play iteration: self-play GPU tests, the self-play bench line, and its kernel-trace summary.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_selfplay_gpu.py tests/test_mcts_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_sp.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload selfplay --no-cpu-baseline > gpurun_out/bench_sp.json 2> gpurun_out/bench_sp.err
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.load(open('gpurun_out/bench_sp.json')); print(d['value'], d['stage_ms_per_sim_step'], d['roofline']['kernel_ms'])"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sp -o sp --output-format csv -- python bench.py --workload selfplay --no-cpu-baseline > gpurun_out/prof_sp.log 2>&1
rc=$?; echo "rocprof rc=$rc"
python - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/prof_sp/sp_kernel_stats.csv')))[:12]:
    print(r['Name'].replace('(anonymous namespace)::', '').split('(')[0][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
exit $rc
